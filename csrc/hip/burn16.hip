// 16x16x32 bf16 MFMA burn, in its own translation unit: it is compiled with
// -mllvm -amdgpu-mfma-vgpr-form (Makefile BURN16_FLAGS) because with AGPR accumulators LLVM rotates
// the eight 4-register chains through v_accvgpr_read/write/mov inside the loop, while the 32x32x16
// burn in kernels.hip keeps its AGPR form (the VGPR form cost it 94 -> 82 % MFMA busy, measured).
#include <hip/hip_runtime.h>

#include "hip_api.h"

namespace gpumon_hip {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Same fragment loader as kernels.hip (32x32x16 layout: A[l&31][8(l>>5)+j], B[8(l>>5)+j][l&31]).
__device__ __forceinline__ void load_frags32(const __bf16* __restrict__ a, const __bf16* __restrict__ b, int lane,
                                             bf16x8* av, bf16x8* bv) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    (*av)[j] = a[r * 16 + 8 * h + j];
    (*bv)[j] = b[(8 * h + j) * 32 + r];
  }
}

// Burn, 16x16x32 form: 8 accumulators x 16 cycles = the same 128 KFLOP per wave per iteration as
// the 32x32x16 loop above, in the shape that holds a higher clock under load on random operands
// (MI355X_MICROARCH.md DVFS item 7: ~1.15x FLOP/s). The register fragments loaded for the 32x32
// form are reused as-is (a burn needs live operands, not a particular product); the 16x16x32
// fragment mapping (A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15], C col l&15 row 4(l>>4)+reg) is what
// the numerics test reproduces.
__global__ void __launch_bounds__(256) mfma_burn16_kernel(const __bf16* __restrict__ a, const __bf16* __restrict__ b,
                                                          float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 av, bv;
  load_frags32(a, b, lane, &av, &bv);
  // named accumulators (an array of vectors made the compiler rotate AGPRs inside the loop)
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {1.f, 0.f, 0.f, 0.f}, c2 = {2.f, 0.f, 0.f, 0.f}, c3 = {3.f, 0.f, 0.f, 0.f};
  f32x4 c4 = {4.f, 0.f, 0.f, 0.f}, c5 = {5.f, 0.f, 0.f, 0.f}, c6 = {6.f, 0.f, 0.f, 0.f}, c7 = {7.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c3, 0, 0, 0);
    c4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c4, 0, 0, 0);
    c5 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c5, 0, 0, 0);
    c6 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c6, 0, 0, 0);
    c7 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, c7, 0, 0, 0);
  }
  const f32x4 t = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  const float s = t[0] + t[1] + t[2] + t[3];
  if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

void launch_mfma_burn16(const __bf16* a, const __bf16* b, float* out, int blocks, int iters, hipStream_t s) {
  hipLaunchKernelGGL(mfma_burn16_kernel, dim3(blocks), dim3(256), 0, s, a, b, out, iters);
}

}  // namespace gpumon_hip
