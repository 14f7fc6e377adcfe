// libgpumon_probe.so — C ABI (ondevice_abi.h) over the K1 gfx950 probe microkernel and its pinned
// ring buffer. Two launch paths share the kernel body (csrc/hip/probe_kernel.h) and the record
// analysis (csrc/hip/probe_collect.h):
//   hsa  raw AQL dispatch of the embedded code object on one HSA queue (probe_hsa.cpp): one
//        hardware queue per GPU, and no HIP runtime in the process;
//   hip  gpumon_hip::Probe (csrc/hip/kernels.hip) on a HIP stream: HIP brings up two queues.
// GPUMON_PROBE_RUNTIME=hsa|hip picks one (default: hsa). The exporter names devices by HIP ordinal
// (hip_id); the HSA path maps it to an agent the way HIP numbers them (hip_to_agent). The exporter binary and gpumon._core dlopen() this library only when the
// probe is enabled, so neither links a GPU runtime.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <vector>

#include "../hip/hip_api.h"
#include "ondevice_abi.h"
#include "probe_hsa.h"

#define GPUMON_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

// HIP's device ordinal -> index among the HSA GPU agents. HIP numbers the agents ROCr exposes (after
// ROCR_VISIBLE_DEVICES) in order, filtered and reordered by HIP_VISIBLE_DEVICES, else
// CUDA_VISIBLE_DEVICES, else GPU_DEVICE_ORDINAL (comma-separated indices). An empty vector means
// "cannot say" (UUID-style entries): the HIP path is used then, so hip_id keeps its meaning.
std::vector<int> hip_to_agent(int n_agents) {
  const char* v = nullptr;
  for (const char* k : {"HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"})
    if ((v = getenv(k)) != nullptr) break;
  std::vector<int> order;
  if (!v) {
    for (int i = 0; i < n_agents; ++i) order.push_back(i);
    return order;
  }
  for (const char* p = v; *p;) {
    while (*p == ' ') ++p;
    char* end = nullptr;
    const long x = strtol(p, &end, 10);
    if (end == p) return {};  // not an index list
    if (x >= 0 && x < n_agents && std::find(order.begin(), order.end(), static_cast<int>(x)) == order.end())
      order.push_back(static_cast<int>(x));
    p = end;
    while (*p == ' ') ++p;
    if (*p == ',') ++p;
    else if (*p) return {};
  }
  return order;
}

struct Runtime {
  bool hsa = false;
  std::vector<int> agent_of;  // hsa: HIP ordinal -> HSA GPU agent index
};

const Runtime& runtime() {
  static const Runtime rt = [] {
    Runtime r;
    const char* e = getenv("GPUMON_PROBE_RUNTIME");
    if (e && !strcmp(e, "hip")) return r;
    r.agent_of = hip_to_agent(gpumon_hsa::gpu_count());
    r.hsa = !r.agent_of.empty() || gpumon_hsa::gpu_count() == 0;
    return r;
  }();
  return rt;
}

bool use_hsa() { return runtime().hsa; }

int agent_of(int hip_dev) {
  const auto& a = runtime().agent_of;
  return hip_dev >= 0 && hip_dev < static_cast<int>(a.size()) ? a[hip_dev] : -1;
}

}  // namespace

struct gpumon_probe {
  std::unique_ptr<gpumon_hip::Probe> p;         // hip
  std::unique_ptr<gpumon_hsa::HsaProbe> hsa;    // hsa
};

GPUMON_EXPORT int gpumon_probe_abi_version(void) { return GPUMON_ONDEVICE_ABI; }

GPUMON_EXPORT int gpumon_probe_device_count(void) {
  return use_hsa() ? static_cast<int>(runtime().agent_of.size()) : gpumon_hip::device_count();
}

// which launch path this process uses ("hsa" / "hip"), for logs and tests
GPUMON_EXPORT const char* gpumon_probe_runtime(void) { return use_hsa() ? "hsa" : "hip"; }

GPUMON_EXPORT size_t gpumon_probe_device_arch(int hip_dev, char* buf, size_t buflen) {
  try {
    std::string a = use_hsa() ? gpumon_hsa::gpu_arch(agent_of(hip_dev)) : gpumon_hip::device_arch(hip_dev);
    if (a.empty()) return 0;
    if (buf && buflen) snprintf(buf, buflen, "%s", a.c_str());
    return a.size() + 1;
  } catch (const std::exception&) {
    return 0;
  }
}

GPUMON_EXPORT size_t gpumon_probe_device_pci(int hip_dev, char* buf, size_t buflen) {
  try {
    std::string a = use_hsa() ? gpumon_hsa::gpu_pci(agent_of(hip_dev)) : gpumon_hip::device_pci_bus_id(hip_dev);
    if (a.empty()) return 0;
    if (buf && buflen) snprintf(buf, buflen, "%s", a.c_str());
    return a.size() + 1;
  } catch (const std::exception&) {
    return 0;
  }
}

GPUMON_EXPORT gpumon_probe* gpumon_probe_create(int hip_dev, int blocks, int slots, int spin_ticks, char* err,
                                                size_t errlen) {
  try {
    auto h = std::make_unique<gpumon_probe>();
    if (use_hsa()) h->hsa = std::make_unique<gpumon_hsa::HsaProbe>(agent_of(hip_dev), blocks, slots, spin_ticks);
    else h->p = std::make_unique<gpumon_hip::Probe>(hip_dev, blocks, slots, spin_ticks);
    return h.release();
  } catch (const std::exception& e) {
    if (err && errlen) snprintf(err, errlen, "%s", e.what());
    return nullptr;
  }
}

GPUMON_EXPORT int gpumon_probe_launch(gpumon_probe* h) {
  if (!h) return -1;
  try {
    return h->hsa ? h->hsa->launch() : h->p->launch();
  } catch (const std::exception&) {
    return -1;
  }
}

GPUMON_EXPORT int gpumon_probe_wait(gpumon_probe* h, int slot, double timeout_s, gpumon_probe_result_t* out) {
  if (!h || !out) return 0;
  gpumon_hip::ProbeResult r;
  bool ok;
  if (h->hsa) ok = timeout_s > 0 ? h->hsa->wait(slot, timeout_s, &r) : h->hsa->poll(slot, &r);
  else ok = timeout_s > 0 ? h->p->wait(slot, timeout_s, &r) : h->p->poll(slot, &r);
  if (!ok) return 0;
  *out = gpumon_probe_result_t{};
  out->seq = r.seq;
  out->blocks = r.blocks;
  out->arrived = r.arrived;
  out->host_latency_s = (r.host_done_ns - r.host_launch_ns) * 1e-9;
  out->gpu_span_s = r.gpu_span_ticks * 1e-8;  // 100 MHz s_memrealtime
  out->unique_cus = r.unique_cus;
  out->wave_slot_mean = r.wave_slot_mean;
  out->stale_records = r.stale_records;
  for (size_t x = 0; x < r.xcc_blocks.size() && x < GPUMON_PROBE_MAX_XCC; ++x) {
    out->xcc_blocks[x] = r.xcc_blocks[x];
    out->xcc_clock_mhz[x] = r.xcc_clock_mhz[x];
    out->xcc_wave_slot[x] = x < r.xcc_wave_slot.size() ? r.xcc_wave_slot[x] : 0.0;
  }
  return 1;
}

GPUMON_EXPORT void gpumon_probe_destroy(gpumon_probe* h) { delete h; }
