// K1 probe device code, shared by the two launch paths:
//   - csrc/hip/kernels.hip   gpumon_hip::probe_kernel, launched through the HIP runtime;
//   - csrc/hip/probe_co.hip  the same body as an unbundled gfx950 code object (extern "C" names),
//                            dispatched as raw AQL packets on one HSA queue
//                            (csrc/plugins/probe_hsa.cpp), so a process that only probes brings
//                            up one hardware queue instead of HIP's two.
// Design notes (publication, wave-slot pressure): kernels.hip, "K1: probe".
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace gpumon_hip {

// One wave per workgroup; the stamps are wave-uniform SGPR reads.
__device__ __forceinline__ void probe_body(ProbeRecord* __restrict__ recs, uint32_t* arrivals, uint32_t* counter,
                                           uint32_t seq, uint32_t spin_ticks, uint32_t blocks) {
  const uint32_t lane = threadIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  uint64_t t1 = t0;
  // Bounded spin on the constant 100 MHz clock: exit condition reached by every wave.
  for (int guard = 0; guard < (1 << 20); ++guard) {
    t1 = __builtin_amdgcn_s_memrealtime();
    if (t1 - t0 >= spin_ticks) break;
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  // ProbeRecord = 3 x 16 B: {xcc_id, hw_id, t0_real}, {t1_real, c0}, {c1, seq, block}
  if (lane < 3) {
    uint4 v;
    if (lane == 0) v = make_uint4(xcc & 0xF, hw, static_cast<uint32_t>(t0), static_cast<uint32_t>(t0 >> 32));
    else if (lane == 1)
      v = make_uint4(static_cast<uint32_t>(t1), static_cast<uint32_t>(t1 >> 32), static_cast<uint32_t>(c0),
                     static_cast<uint32_t>(c0 >> 32));
    else v = make_uint4(static_cast<uint32_t>(c1), static_cast<uint32_t>(c1 >> 32), seq, blockIdx.x);
    reinterpret_cast<uint4*>(recs + blockIdx.x)[lane] = v;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == blocks - 1) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm the slot
      __hip_atomic_store(arrivals, blocks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace gpumon_hip
