// Fake on-device plugins (both C ABIs of csrc/plugins/ondevice_abi.h) for CPU tests of the native
// PMC / probe samplers (csrc/core/ondevice.cpp) through the same dlopen path the exporter uses on a
// GPU node. Built twice, as build/fakes/ondevice/libgpumon_pmc.so and libgpumon_probe.so.
//
// Scripted by environment:
//   GPUMON_FAKE_AGENTS      GPU agents / HIP devices (default 1)
//   GPUMON_FAKE_MFMA        MFMA busy fraction 0..1 (default 0.5), spread evenly over 8 XCCs
//   GPUMON_FAKE_OCC         occupancy fraction 0..1 (default 0.25)
//   GPUMON_FAKE_TFLOPS      bf16 MFMA TFLOP/s (default 1000; f16 at a tenth, other types 0)
//   GPUMON_FAKE_PMC_FAIL    "init" -> init fails; "sample" -> every sample reports not-ok;
//                           "start" -> continuous counting cannot start (counters held elsewhere)
//   GPUMON_FAKE_PMC_READ    continuous reads: "cumulative" (default: values since the start) or
//                           "reset" (values since the previous read)
//   GPUMON_FAKE_PMC_RESTART every Nth continuous read the counts restart from 0 without the
//                           started flag (another tool restarted the contexts underneath)
//   GPUMON_FAKE_PROBE_HANG  1 -> launches never complete (timeouts path)
//   GPUMON_FAKE_DEAD_XCD    N -> no probe workgroup runs on XCD N (liveness path)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <chrono>

#include "../plugins/ondevice_abi.h"

#define EXPORT extern "C" __attribute__((visibility("default")))

namespace {
int agents() {
  const char* e = getenv("GPUMON_FAKE_AGENTS");
  return e ? atoi(e) : 1;
}
double envd(const char* k, double d) {
  const char* e = getenv(k);
  return e ? atof(e) : d;
}
bool fail(const char* what) {
  const char* e = getenv("GPUMON_FAKE_PMC_FAIL");
  return e && strcmp(e, what) == 0;
}
constexpr uint32_t kCus = 256, kSimds = 1024, kXcc = 8, kWaves = 32;
constexpr double kClock = 2.4e9;
}  // namespace

EXPORT int gpumon_pmc_abi_version(void) { return GPUMON_ONDEVICE_ABI; }

EXPORT int gpumon_pmc_init(char* err, size_t errlen) {
  if (fail("init")) {
    snprintf(err, errlen, "fake: device counting unavailable");
    return -1;
  }
  return agents();
}

EXPORT int gpumon_pmc_agent(int agent, gpumon_pmc_agent_t* out) {
  if (agent < 0 || agent >= agents() || !out) return -1;
  *out = gpumon_pmc_agent_t{};
  out->node_id = 2 + agent;
  out->logical_node_id = 1 + agent;
  out->drm_render_minor = 128 + agent;
  out->cu_count = kCus;
  out->simd_count = kSimds;
  out->num_xcc = kXcc;
  out->max_waves_per_cu = kWaves;
  snprintf(out->name, sizeof out->name, "gfx950");
  snprintf(out->product_name, sizeof out->product_name, "fake MI355X");
  return 0;
}

EXPORT size_t gpumon_pmc_supported(int, char* buf, size_t n) {
  const char* s =
      "GRBM_COUNT\nGRBM_GUI_ACTIVE\nSQ_VALU_MFMA_BUSY_CYCLES\nSQ_WAVE_CYCLES\nSQ_INSTS_VALU_MFMA_MOPS_BF16\n"
      "SQ_INSTS_VALU_MFMA_MOPS_F16\nSQ_INSTS_VALU_MFMA_MOPS_F8\nSQ_INSTS_VALU_MFMA_MOPS_F6F4\n"
      "SQ_INSTS_VALU_MFMA_MOPS_F32\nSQ_INSTS_VALU_MFMA_MOPS_F64\nSQ_INSTS_VALU_MFMA_MOPS_I8\n";
  if (buf && n) snprintf(buf, n, "%s", s);
  return strlen(s) + 1;
}

EXPORT size_t gpumon_pmc_dimensions(int, const char*, char* buf, size_t n) {
  const char* s = "DIMENSION_XCC:8\n";
  if (buf && n) snprintf(buf, n, "%s", s);
  return strlen(s) + 1;
}

namespace {
// Values of `counters` for a counting span of window_s seconds (both sampling modes use it).
int fill(int n_agents, const char* const* counters, int n_counters, double window_s, gpumon_pmc_value_t* out,
         int32_t* ok, char* err, size_t errlen) {
  const double gui = window_s * kClock;
  for (int k = 0; k < n_agents; ++k) {
    ok[k] = fail("sample") ? 0 : 1;
    for (int c = 0; c < n_counters; ++c) {
      gpumon_pmc_value_t& v = out[k * n_counters + c];
      v = gpumon_pmc_value_t{};
      if (!ok[k]) continue;
      std::string name = counters[c];
      double total = 0;
      bool per_xcc = true;
      if (name == "GRBM_GUI_ACTIVE" || name == "GRBM_COUNT") {
        total = gui;
        per_xcc = false;
      } else if (name == "SQ_VALU_MFMA_BUSY_CYCLES") {
        total = envd("GPUMON_FAKE_MFMA", 0.5) * gui * kSimds;
      } else if (name == "SQ_WAVE_CYCLES") {
        total = envd("GPUMON_FAKE_OCC", 0.25) * gui * kCus * kWaves / 4.0;
      } else if (name.rfind("SQ_INSTS_VALU_MFMA_MOPS_", 0) == 0) {
        const double tf = envd("GPUMON_FAKE_TFLOPS", 1000.0);
        const std::string dt = name.substr(24);
        total = (dt == "BF16" ? tf : dt == "F16" ? tf / 10 : 0.0) * 1e12 * window_s / 512.0;
      } else {
        snprintf(err, errlen, "counter not supported: %s", name.c_str());
        return -1;
      }
      v.ok = 1;
      if (per_xcc) {
        v.n = kXcc;
        v.n_xcc = kXcc;
        for (uint32_t x = 0; x < kXcc; ++x) v.by_xcc[x] = total / kXcc;
        v.sum = total;
        v.max = total / kXcc;
      } else {
        v.n = kXcc;  // GRBM is replicated per XCC: max is the device value
        v.sum = total * kXcc;
        v.max = total;
      }
    }
  }
  return 0;
}

bool g_running = false;
std::chrono::steady_clock::time_point g_t0, g_last;
}  // namespace

EXPORT int gpumon_pmc_sample_many(const int* ags, int n_agents, const char* const* counters, int n_counters,
                                  double window_s, gpumon_pmc_value_t* out, int32_t* ok, char* err, size_t errlen) {
  for (int k = 0; k < n_agents; ++k)
    if (ags[k] < 0 || ags[k] >= agents()) {
      snprintf(err, errlen, "pmc agent index");
      return -1;
    }
  g_running = false;
  std::this_thread::sleep_for(std::chrono::duration<double>(window_s));
  return fill(n_agents, counters, n_counters, window_s, out, ok, err, errlen);
}

EXPORT int gpumon_pmc_read_running(const int* ags, int n_agents, const char* const* counters, int n_counters,
                                   gpumon_pmc_value_t* out, int32_t* ok, int32_t* started, char* err, size_t errlen) {
  for (int k = 0; k < n_agents; ++k)
    if (ags[k] < 0 || ags[k] >= agents()) {
      snprintf(err, errlen, "pmc agent index");
      return -1;
    }
  const auto now = std::chrono::steady_clock::now();
  if (started) *started = 0;
  if (!g_running) {
    if (fail("start")) {
      snprintf(err, errlen, "pmc read: start_context failed on agent %d (another profiler holds the device counters?)",
               ags[0]);
      return -1;
    }
    g_running = true;
    g_t0 = g_last = now;
    if (started) *started = 1;
  }
  static int reads = 0;
  const int restart = static_cast<int>(envd("GPUMON_FAKE_PMC_RESTART", 0));
  if (restart > 0 && ++reads % restart == 0) g_t0 = now - std::chrono::milliseconds(1);
  const char* mode = getenv("GPUMON_FAKE_PMC_READ");
  const bool reset = mode && strcmp(mode, "reset") == 0;
  const double span = std::chrono::duration<double>(now - (reset ? g_last : g_t0)).count();
  g_last = now;
  return fill(n_agents, counters, n_counters, span, out, ok, err, errlen);
}

EXPORT void gpumon_pmc_stop_running(void) { g_running = false; }

// ---- probe ----------------------------------------------------------------------------------
struct gpumon_probe {
  int dev;
  int blocks;
  uint32_t seq;
};

EXPORT int gpumon_probe_abi_version(void) { return GPUMON_ONDEVICE_ABI; }
EXPORT int gpumon_probe_device_count(void) { return agents(); }
// PCI address per HIP ordinal from GPUMON_FAKE_PCI ("0000:65:00.0,0000:a5:00.0": a
// HIP_VISIBLE_DEVICES-style subset of the mock's GPUs); unset = unknown, the exporter pairs by hip_id
EXPORT size_t gpumon_probe_device_pci(int dev, char* buf, size_t n) {
  const char* v = getenv("GPUMON_FAKE_PCI");
  if (!v || dev < 0 || dev >= agents()) return 0;
  char b[32];
  const char* p = v;
  for (int k = 0; k < dev && p; ++k) {
    p = strchr(p, ',');
    if (p) ++p;
  }
  if (!p || !*p) return 0;
  const size_t len = strcspn(p, ",");
  if (len >= sizeof b) return 0;
  memcpy(b, p, len);
  b[len] = 0;
  if (buf && n) snprintf(buf, n, "%s", b);
  return strlen(b) + 1;
}
EXPORT size_t gpumon_probe_device_arch(int, char* buf, size_t n) {
  if (buf && n) snprintf(buf, n, "gfx950:sramecc+:xnack-");
  return 23;
}
EXPORT gpumon_probe* gpumon_probe_create(int dev, int blocks, int, int, char* err, size_t errlen) {
  if (dev < 0 || dev >= agents()) {
    snprintf(err, errlen, "fake: no hip device %d", dev);
    return nullptr;
  }
  return new gpumon_probe{dev, blocks, 0};
}
EXPORT int gpumon_probe_launch(gpumon_probe* p) { return p ? static_cast<int>(p->seq++ % 4) : -1; }
EXPORT int gpumon_probe_wait(gpumon_probe* p, int, double timeout_s, gpumon_probe_result_t* out) {
  if (!p || !out) return 0;
  if (getenv("GPUMON_FAKE_PROBE_HANG")) {
    std::this_thread::sleep_for(std::chrono::duration<double>(timeout_s));
    return 0;
  }
  *out = gpumon_probe_result_t{};
  out->seq = p->seq;
  out->blocks = p->blocks;
  out->arrived = p->blocks;
  out->host_latency_s = 25e-6;
  out->gpu_span_s = 6e-6;
  out->unique_cus = kCus;
  out->wave_slot_mean = 1.75;
  const char* dead = getenv("GPUMON_FAKE_DEAD_XCD");
  for (uint32_t x = 0; x < kXcc; ++x) {
    out->xcc_blocks[x] = dead && static_cast<uint32_t>(atoi(dead)) == x ? 0 : p->blocks / kXcc;
    out->xcc_clock_mhz[x] = 2400.0 - 10.0 * x;
    out->xcc_wave_slot[x] = 0.5 * x;
  }
  return 1;
}
EXPORT void gpumon_probe_destroy(gpumon_probe* p) { delete p; }
