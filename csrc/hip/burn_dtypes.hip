// MFMA burns per operand type, to validate gpu_mfma_tflops{dtype} (the per-type
// SQ_INSTS_VALU_MFMA_MOPS_* counters) against event-timed FLOPs and to characterise what each
// gfx950 matrix path sustains. Same shape as the 16x16x32 bf16 burn (burn16.hip): 256-thread
// workgroups, 8 independent accumulator chains per wave, operands fixed in registers (a burn needs
// live operands, not a particular product), compiled with VGPR-form accumulators (Makefile).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "hip_api.h"

namespace gpumon_hip {

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

enum Kind { kF16 = 0, kFp8, kF32, kF64, kI8, kMxFp8, kMxFp4 };

// One MFMA of each kind on accumulator c (operands a/b already in registers).
template <int K>
struct Op;
template <>
struct Op<kF16> {
  using Acc = f32x4;
  static constexpr double kFlop = 2.0 * 16 * 16 * 32;
  __device__ static Acc run(Acc c, int lane) {
    f16x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = static_cast<_Float16>(0.5f + 0.001f * ((lane + j) & 7));
      b[j] = static_cast<_Float16>(0.25f);
    }
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <>
struct Op<kFp8> {
  using Acc = f32x4;
  static constexpr double kFlop = 2.0 * 16 * 16 * 32;
  __device__ static Acc run(Acc c, int lane) {
    const long a = 0x3838383838383838L + (lane & 1), b = 0x3030303030303030L;  // e4m3 1.0 / 0.5
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
  }
};
template <>
struct Op<kF32> {
  using Acc = f32x4;
  static constexpr double kFlop = 2.0 * 16 * 16 * 4;
  __device__ static Acc run(Acc c, int lane) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(1.0f + lane * 1e-3f, 0.5f, c, 0, 0, 0);
  }
};
template <>
struct Op<kF64> {
  using Acc = f64x4;
  static constexpr double kFlop = 2.0 * 16 * 16 * 4;
  __device__ static Acc run(Acc c, int lane) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(1.0 + lane * 1e-3, 0.5, c, 0, 0, 0);
  }
};
template <>
struct Op<kI8> {
  using Acc = i32x4;
  static constexpr double kFlop = 2.0 * 16 * 16 * 64;  // integer ops
  __device__ static Acc run(Acc c, int lane) {
    const i32x4 a = {0x01010101 + (lane & 1), 0x01010101, 0x01010101, 0x01010101};
    const i32x4 b = {0x02020202, 0x02020202, 0x02020202, 0x02020202};
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  }
};
template <>
struct Op<kMxFp8> {  // block-scaled f8f6f4 path, fp8 (e4m3) operands, unit scales
  using Acc = f32x4;
  static constexpr double kFlop = 2.0 * 16 * 16 * 128;
  __device__ static Acc run(Acc c, int lane) {
    i32x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = 0x38383838 + ((lane + j) & 1);
      b[j] = 0x30303030;
    }
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
  }
};
template <>
struct Op<kMxFp4> {  // block-scaled f8f6f4 path, fp4 (e2m1) operands, unit scales
  using Acc = f32x4;
  static constexpr double kFlop = 2.0 * 16 * 16 * 128;
  __device__ static Acc run(Acc c, int lane) {
    i32x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = 0x22222222 + ((lane + j) & 1);  // e2m1 1.0 nibbles
      b[j] = 0x11111111;                     // e2m1 0.5
    }
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
  }
};

template <int K>
__global__ void __launch_bounds__(256) burn_kernel(float* __restrict__ out, int iters) {
  using Acc = typename Op<K>::Acc;
  const int lane = threadIdx.x & 63;
  Acc c0 = {}, c1 = {}, c2 = {}, c3 = {}, c4 = {}, c5 = {}, c6 = {}, c7 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = Op<K>::run(c0, lane);
    c1 = Op<K>::run(c1, lane);
    c2 = Op<K>::run(c2, lane);
    c3 = Op<K>::run(c3, lane);
    c4 = Op<K>::run(c4, lane);
    c5 = Op<K>::run(c5, lane);
    c6 = Op<K>::run(c6, lane);
    c7 = Op<K>::run(c7, lane);
  }
  const Acc t = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = static_cast<float>(t[0] + t[1] + t[2] + t[3]);
}

template <int K>
double launch(float* out, int blocks, int iters, hipStream_t s) {
  hipLaunchKernelGGL(burn_kernel<K>, dim3(blocks), dim3(256), 0, s, out, iters);
  return static_cast<double>(blocks) * 4 * 8 * iters * Op<K>::kFlop;
}
}  // namespace

double launch_mfma_burn_dtype(int dev, const std::string& dtype, float* out, int blocks, int iters, void* stream) {
  check(hipSetDevice(dev), "hipSetDevice");
  auto s = static_cast<hipStream_t>(stream);
  double flop;
  if (dtype == "f16") flop = launch<kF16>(out, blocks, iters, s);
  else if (dtype == "fp8") flop = launch<kFp8>(out, blocks, iters, s);
  else if (dtype == "f32") flop = launch<kF32>(out, blocks, iters, s);
  else if (dtype == "f64") flop = launch<kF64>(out, blocks, iters, s);
  else if (dtype == "i8") flop = launch<kI8>(out, blocks, iters, s);
  else if (dtype == "mxfp8") flop = launch<kMxFp8>(out, blocks, iters, s);
  else if (dtype == "mxfp4") flop = launch<kMxFp4>(out, blocks, iters, s);
  else throw std::invalid_argument("mfma_burn_dtype: dtype must be f16|fp8|f32|f64|i8|mxfp8|mxfp4");
  check(hipGetLastError(), "burn_kernel");
  return flop;
}

}  // namespace gpumon_hip
