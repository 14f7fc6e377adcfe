// C ABI of the two on-device plugins the exporter dlopen()s at run time:
//
//   lib/libgpumon_pmc.so    rocprofiler-sdk device counting (SQ/GRBM PMCs, whole GPU, host thread)
//   lib/libgpumon_probe.so  the K1 gfx950 probe microkernel + its pinned ring buffer (raw HSA / AQL;
//                           HIP with GPUMON_PROBE_RUNTIME=hip)
//
// Why plugins: bin/gpumon-exporter links neither HIP nor rocprofiler-sdk, so the same binary runs
// on a node without them and only pays for them when --pmc / --probe ask (the SURVEY N1 role: the
// agent is decoupled from the host's tool-library ABI, like the reference's libltdl.so.7). The
// Python modules gpumon._pmc / gpumon._hip and the C++ samplers (csrc/core/ondevice.cpp) use the
// same code, so there is one implementation of each on-device path.
//
// All functions are thread-compatible, not thread-safe per handle: one sampler thread owns a probe.
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPUMON_ONDEVICE_ABI 3  // 2: gpumon_probe_result_t.stale_records + xcc_wave_slot; 3: continuous PMC reads
#define GPUMON_PMC_MAX_XCC 16

// ---- PMC (libgpumon_pmc.so) --------------------------------------------------------------------
typedef struct {
  uint32_t node_id;
  uint32_t logical_node_id;
  int32_t drm_render_minor;
  uint32_t cu_count;
  uint32_t simd_count;
  uint32_t num_xcc;
  uint32_t max_waves_per_cu;
  char name[64];
  char product_name[64];
} gpumon_pmc_agent_t;

typedef struct {
  int32_t ok;       // 1 when the counter produced records in this window
  double sum;       // over every dimension instance
  double max;
  uint64_t n;       // instances
  int32_t n_xcc;    // entries of by_xcc (0 if the counter has no XCC dimension)
  double by_xcc[GPUMON_PMC_MAX_XCC];
} gpumon_pmc_value_t;

int gpumon_pmc_abi_version(void);
// Registers the tool (rocprofiler_force_configure) and brings HSA up. Must run before anything
// else initialises HSA/HIP in the process. Returns the GPU agent count, or -1 with `err` set.
int gpumon_pmc_init(char* err, size_t errlen);
int gpumon_pmc_agent(int agent, gpumon_pmc_agent_t* out);
// Names of the counters the agent supports, '\n'-separated; returns the bytes needed (incl. NUL).
size_t gpumon_pmc_supported(int agent, char* buf, size_t buflen);
// Dimensions of one counter as "NAME:instances\n" lines; returns bytes needed, 0 if unsupported.
size_t gpumon_pmc_dimensions(int agent, const char* counter, char* buf, size_t buflen);
// Every listed agent counts over ONE shared window of `window_s` seconds. out[a * n_counters + c];
// ok[a] = 1 for agents whose sample succeeded. Returns 0, or -1 with `err` set (bad counter name /
// agent index; nothing was sampled).
int gpumon_pmc_sample_many(const int* agents, int n_agents, const char* const* counters, int n_counters,
                           double window_s, gpumon_pmc_value_t* out, int32_t* ok, char* err, size_t errlen);
// Continuous counting: the contexts stay started between calls, each call reads them without a
// stop (no uncounted gap between reads). The first call, or one with a different request, (re)starts
// them and sets *started = 1. A gpumon_pmc_sample_many call ends continuous counting.
int gpumon_pmc_read_running(const int* agents, int n_agents, const char* const* counters, int n_counters,
                            gpumon_pmc_value_t* out, int32_t* ok, int32_t* started, char* err, size_t errlen);
void gpumon_pmc_stop_running(void);

// ---- K1 probe (libgpumon_probe.so) -------------------------------------------------------------
typedef struct gpumon_probe gpumon_probe;

#define GPUMON_PROBE_MAX_XCC 16
typedef struct {
  uint32_t seq;
  int32_t blocks;
  int32_t arrived;
  double host_latency_s;   // host launch -> last arrival observed
  double gpu_span_s;       // max(end) - min(start) on the 100 MHz clock
  int32_t unique_cus;
  int32_t stale_records;   // records not yet visible when the arrival flag was (expected 0)
  int32_t xcc_blocks[GPUMON_PROBE_MAX_XCC];
  double xcc_clock_mhz[GPUMON_PROBE_MAX_XCC];
  // Mean over the SIMDs a launch landed on of the lowest wave slot (HW_ID.WAVE_ID) a probe wave got
  // there: the wave slots already held by other work at launch time (0 on an idle XCD).
  double xcc_wave_slot[GPUMON_PROBE_MAX_XCC];
  double wave_slot_mean;
} gpumon_probe_result_t;

int gpumon_probe_abi_version(void);
int gpumon_probe_device_count(void);
// Arch string of a HIP device ("gfx950:sramecc+:xnack-"), bytes needed incl. NUL.
size_t gpumon_probe_device_arch(int hip_dev, char* buf, size_t buflen);
// Optional: PCI address of a HIP device ("0000:75:00.0"), bytes needed incl. NUL (0: unknown). The
// exporter pairs its devices with the helper's HIP ordinals by it: the helper's ordinals follow
// HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES, the exporter's hip_id does not.
size_t gpumon_probe_device_pci(int hip_dev, char* buf, size_t buflen);
gpumon_probe* gpumon_probe_create(int hip_dev, int blocks, int slots, int spin_ticks, char* err, size_t errlen);
int gpumon_probe_launch(gpumon_probe* p);  // slot >= 0, or -1 when every slot is still in flight
// 1 = complete (result filled), 0 = not yet (after waiting up to timeout_s; 0 = just poll)
int gpumon_probe_wait(gpumon_probe* p, int slot, double timeout_s, gpumon_probe_result_t* out);
void gpumon_probe_destroy(gpumon_probe* p);

#ifdef __cplusplus
}
#endif
