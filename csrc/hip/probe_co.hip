// The K1 probe as a stand-alone gfx950 code object (built unbundled with --offload-device-only, and
// embedded in lib/libgpumon_probe.so): the raw-HSA launch path (csrc/plugins/probe_hsa.cpp) loads
// it into an hsa_executable and dispatches AQL packets itself, without the HIP runtime.
// extern "C" keeps the symbol names stable: gpumon_probe_kernel.kd / gpumon_probe_reset.kd.
#include "probe_kernel.h"

using gpumon_hip::ProbeRecord;

// Kernel argument layout (checked against the code object's metadata by tests/test_probe_hsa.py):
//   0 recs (8), 8 arrivals (8), 16 counters (8), 24 seq (4), 28 spin_ticks (4), 32 blocks (4) = 36 B
extern "C" __global__ void __launch_bounds__(64) gpumon_probe_kernel(ProbeRecord* __restrict__ recs,
                                                                     uint32_t* arrivals, uint32_t* counter,
                                                                     uint32_t seq, uint32_t spin_ticks,
                                                                     uint32_t blocks) {
  gpumon_hip::probe_body(recs, arrivals, counter, seq, spin_ticks, blocks);
}

// Zeroes the per-slot arrival counters in device memory once, before the first probe launch (the
// HIP path used hipMemsetAsync; here a copy engine or blit kernel would bring up another queue).
//   0 counters (8), 8 n (4) = 12 B; one 64-lane workgroup, grid-stride.
extern "C" __global__ void __launch_bounds__(64) gpumon_probe_reset(uint32_t* counters, uint32_t n) {
  for (uint32_t i = threadIdx.x; i < n; i += 64)
    __hip_atomic_store(counters + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
