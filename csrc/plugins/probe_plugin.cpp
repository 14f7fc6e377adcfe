// libgpumon_probe.so — C ABI (ondevice_abi.h) over the K1 gfx950 probe microkernel and its pinned
// ring buffer (gpumon_hip::Probe, csrc/hip/kernels.hip). Linked with kernels.o by hipcc; the
// exporter binary and gpumon._core dlopen() it only when the probe is enabled, so neither links the
// HIP runtime.
#include <cstdio>
#include <exception>
#include <memory>
#include <string>

#include "../hip/hip_api.h"
#include "ondevice_abi.h"

#define GPUMON_EXPORT extern "C" __attribute__((visibility("default")))

struct gpumon_probe {
  std::unique_ptr<gpumon_hip::Probe> p;
};

GPUMON_EXPORT int gpumon_probe_abi_version(void) { return GPUMON_ONDEVICE_ABI; }

GPUMON_EXPORT int gpumon_probe_device_count(void) { return gpumon_hip::device_count(); }

GPUMON_EXPORT size_t gpumon_probe_device_arch(int hip_dev, char* buf, size_t buflen) {
  try {
    std::string a = gpumon_hip::device_arch(hip_dev);
    if (buf && buflen) snprintf(buf, buflen, "%s", a.c_str());
    return a.size() + 1;
  } catch (const std::exception&) {
    return 0;
  }
}

GPUMON_EXPORT gpumon_probe* gpumon_probe_create(int hip_dev, int blocks, int slots, int spin_ticks, char* err,
                                                size_t errlen) {
  try {
    auto* h = new gpumon_probe;
    h->p = std::make_unique<gpumon_hip::Probe>(hip_dev, blocks, slots, spin_ticks);
    return h;
  } catch (const std::exception& e) {
    if (err && errlen) snprintf(err, errlen, "%s", e.what());
    return nullptr;
  }
}

GPUMON_EXPORT int gpumon_probe_launch(gpumon_probe* h) {
  if (!h) return -1;
  try {
    return h->p->launch();
  } catch (const std::exception&) {
    return -1;
  }
}

GPUMON_EXPORT int gpumon_probe_wait(gpumon_probe* h, int slot, double timeout_s, gpumon_probe_result_t* out) {
  if (!h || !out) return 0;
  gpumon_hip::ProbeResult r;
  const bool ok = timeout_s > 0 ? h->p->wait(slot, timeout_s, &r) : h->p->poll(slot, &r);
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
