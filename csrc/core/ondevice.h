// On-device samplers of the native exporter: rocprofiler-sdk device counting (MFMA busy /
// occupancy) and the K1 gfx950 probe microkernel, each in its own thread, publishing through
// Exporter::set_extra() like every other out-of-band source.
//
// Neither is linked: both live in plugins (csrc/plugins/ondevice_abi.h) that this file dlopen()s
// from <dir of this binary or .so>/../lib, or GPUMON_PLUGIN_DIR. The exporter binary therefore
// runs on a node without HIP or rocprofiler-sdk and only loads them when --pmc / --probe ask — the
// role the reference gives its vendored libltdl.so.7 (/root/reference/Dockerfile:4):
// keep the agent independent of the host's tool-library ABI.
//
// Production placement (ondevice_isolate, the default): both plugins run in ONE child process,
// lib/gpumon-ondevice-helper, driven over a pipe pair (csrc/plugins/ondevice_helper_proto.h) and
// SIGSTOPped between requests. rocprofiler-sdk's device counting leaves an HSA thread polling a
// full core in the process that owns it; a frozen process polls nothing, the counters keep
// counting, and this process never maps HIP, HSA or rocprofiler-sdk. A probe step is one request
// (launch + wait in one awake period), a dead helper is respawned with backoff (PMC re-initialised
// before any probe op: rocprofiler must register before HSA comes up), and the helper's CPU and
// RSS are exported because they are part of the pod's footprint (profiles/r2_footprint.md).
//
// Series and formulas match tests/oracles/ops/pmc.py and tests/oracles/ops/probe.py (the Python test oracles
// under tests/oracles, not shipped), so dashboards see the same families from either path. The PMC
// sampler also publishes each GPU's MFMA utilisation to the exporter for pod_gpu_mfma_util_percent.
#pragma once

#include <atomic>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "render.h"
#include "sample.h"

namespace gpumon {

class Exporter;

struct OnDeviceConfig {
  std::string plugin_dir;   // "" = $GPUMON_PLUGIN_DIR or <dir of this object>/../lib
  bool pmc = false;
  // MFMA busy + MFMA MOPS per operand type + GRBM: 8 SQ + 2 GRBM = one gfx950 counting pass. No
  // per-wave SQ counters: they count only the profiling process's waves (tests/oracles/ops/pmc.py).
  std::vector<std::string> pmc_counters = {
      "SQ_VALU_MFMA_BUSY_CYCLES",    "SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_INSTS_VALU_MFMA_MOPS_F16",
      "SQ_INSTS_VALU_MFMA_MOPS_F8",  "SQ_INSTS_VALU_MFMA_MOPS_F6F4", "SQ_INSTS_VALU_MFMA_MOPS_F32",
      "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_INSTS_VALU_MFMA_MOPS_I8",   "GRBM_GUI_ACTIVE",
      "GRBM_COUNT"};
  double pmc_every_s = 1.0;
  // "continuous": the counting contexts run all the time and every step reads them without a stop
  // (cumulative counts, measured on MI355X: profiles/r2_pmc_continuous.md), so 100 % of each
  // interval is counted; "window": start -> pmc_window_s -> read -> stop per step (the r1 sampler:
  // aliases bursts longer than the window). Continuous falls back to window when the plugin lacks it.
  std::string pmc_mode = "continuous";
  // true: the device counting contexts and the K1 probe run in <plugin dir>/gpumon-ondevice-helper,
  // a child process frozen between requests (rocprofiler-sdk leaves an HSA thread polling a full
  // core in the process that owns the contexts; this process then never loads a GPU runtime);
  // false: the plugins in this process (tools that already run HIP / HSA).
  bool ondevice_isolate = true;
  double helper_retry_s = 10.0;  // a dead helper is respawned at most this often
  double pmc_window_s = 0.1;  // window mode: counting window per sample (capped at half the period)
  bool probe = false;
  double probe_every_s = 1.0;
  int probe_blocks = 1024;    // one-wave workgroups per launch (>= 4 per CU spreads over all 8 XCDs)
  int probe_spin_ticks = 200;
  double probe_timeout_s = 0.5;
};

// Reduced counter values of one agent (sum / max over instances, per-XCC sums).
struct PmcReduced {
  double sum = 0, max = 0;
  uint64_t n = 0;
  std::vector<double> by_xcc;
};

struct PmcAgentInfo {
  uint32_t cu_count = 0, simd_count = 0, num_xcc = 0, max_waves_per_cu = 0;
  int drm_render_minor = -1;
};

// NaN = not derivable from the counters given.
struct PmcDerived {
  // mfma_busy: MFMA busy cycles as a share of the GPU's ACTIVE cycles (GRBM_GUI_ACTIVE x SIMDs);
  // mfma_util: the same as a share of WALL time (x the firmware's wall-time gfx activity, set by
  // OnDevice); gui_active: active cycles / all cycles (GRBM_COUNT slows while idle: a cycle share).
  double mfma_busy = kNaN, mfma_util = kNaN, occupancy = kNaN, gui_active = kNaN;
  std::vector<double> xcd_mfma_busy, xcd_mfma_util;
  double span_s = 0;      // counted time behind this sample
  double coverage = kNaN; // counted time / wall time since the previous sample
  std::vector<std::pair<std::string, double>> mfma_tflops;  // (dtype lower-case, TFLOP/s), by name
};

// Pure (CPU-tested against tests/oracles/ops/pmc.py derive): the gfx9xx formulas ROCm 7.2 falls back to on gfx950.
// window_s > 0 adds the MFMA TFLOP/s per operand type (512 FLOP per SQ_INSTS_VALU_MFMA_MOPS_* unit).
PmcDerived pmc_derive(const std::map<std::string, PmcReduced>& raw, const PmcAgentInfo& agent, double window_s = 0);

// Directory the plugins are looked up in (see OnDeviceConfig::plugin_dir).
std::string default_plugin_dir();

class OnDevice {
 public:
  OnDevice(Exporter* ex, OnDeviceConfig cfg);
  ~OnDevice();
  // Loads and initialises the enabled plugins (PMC before the probe: rocprofiler must register before
  // the HIP runtime initialises HSA) and starts their threads. False + err when a requested plugin
  // cannot be loaded; nothing is left running then.
  bool start(std::string* err);
  void stop();
  // One synchronous step of each enabled sampler (tests, --once); returns false if none is enabled.
  bool step();

  struct Stats {
    uint64_t pmc_samples = 0, pmc_errors = 0, pmc_resets = 0, probe_done = 0, probe_timeouts = 0;
    uint64_t pmc_steps = 0, probe_steps = 0;  // steps begun (the sampler threads' and synchronous ones)
    uint64_t helper_restarts = 0;
    int pmc_agents = 0, probe_devices = 0;
    bool probe_by_bdf = false;
    bool pmc_continuous = false;
  };
  Stats stats() const;

  struct Plugin;  // dlopen'd function table (ondevice.cpp)

 private:
  void pmc_loop();
  void probe_loop();
  void pmc_step();
  void pmc_step_window(const std::vector<int>& devs, const std::vector<int>& ags);
  void pmc_step_continuous(const std::vector<int>& devs, const std::vector<int>& ags);
  void finish_derived(int dev, PmcDerived* d);
  void probe_step();
  void map_pmc_agents();
  bool create_probes(std::string* err);
  void export_pmc();
  void export_probe();
  void sleep_until(int64_t deadline_ns);
  // ondevice_isolate: true when the helper is up; a dead helper (crashed, OOM-killed) is respawned
  // and re-initialised here, at most once per helper_retry_s, by whichever sampler notices first
  bool helper_check();
  void export_helper();

  Exporter* ex_;
  OnDeviceConfig cfg_;
  std::unique_ptr<Plugin> pmc_lib_, probe_lib_;

  std::mutex pmc_mu_, probe_mu_;
  std::vector<PmcAgentInfo> agents_;
  std::map<int, int> pmc_map_;  // exporter device index -> pmc agent index
  std::map<int, PmcDerived> pmc_last_;
  // continuous mode: the previous read per device and when it was taken
  std::map<int, std::map<std::string, PmcReduced>> pmc_prev_;
  int64_t pmc_prev_ns_ = 0;
  bool pmc_continuous_ = false;
  bool helper_ = false;         // pmc_lib_ / probe_lib_ are clients of the helper process
  std::string helper_path_;
  std::mutex recover_mu_;       // helper respawn + PMC re-init (before any probe op on a new helper)
  int64_t next_respawn_ns_ = 0;
  int64_t helper_spawned_ns_ = 0;  // when the current helper was (re)spawned
  int respawn_streak_ = 0;          // respawns of helpers that died within 10 minutes (backoff)
  std::atomic<uint64_t> helper_gen_{0}, helper_restarts_{0};
  uint64_t probe_gen_seen_ = 0;  // helper generation the probe handles belong to
  int64_t pmc_last_ok_ns_ = 0;  // last step that produced values (window or continuous)
  bool pmc_up_ = false;

  struct ProbeDev {
    int dev = 0;
    void* handle = nullptr;
    int pending = -1;   // slot in flight, -1 none
    uint64_t timeouts = 0;
    uint64_t stale = 0;     // records that had not landed when the arrival flag had
    bool have = false;
    double latency_s = 0, span_s = 0;
    int unique_cus = 0;
    std::vector<int> xcc_blocks;
    std::vector<double> xcc_mhz;
    std::vector<double> xcc_slot;
    double slot_mean = 0;
  };
  std::vector<ProbeDev> probes_;
  bool probe_by_bdf_ = false;  // probes paired with exporter devices by PCI address (else hip_id)

  std::atomic<bool> running_{false};
  std::atomic<bool> stopped_{false};
  std::mutex wait_mu_;
  std::condition_variable wait_cv_;
  std::thread pmc_th_, probe_th_;
  std::atomic<uint64_t> pmc_samples_{0}, pmc_errors_{0}, pmc_resets_{0}, probe_done_{0}, probe_timeouts_{0};
  std::atomic<uint64_t> pmc_steps_{0}, probe_steps_{0};
};

// pid of the on-device helper process this exporter spawned (0: none running). Its GPU context
// (PMC counting buffers, the K1 probe's waves) is the exporter's own, not a workload's.
int ondevice_helper_pid();

}  // namespace gpumon
