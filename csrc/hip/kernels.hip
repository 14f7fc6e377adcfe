// gfx950 kernels + host wrappers. See kernels.h for the design notes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <stdexcept>
#include <tuple>

#include "hip_api.h"
#include "probe_kernel.h"

namespace gpumon_hip {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

static int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void check(int err, const char* what) {
  if (err != hipSuccess)
    throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(static_cast<hipError_t>(err)));
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

std::string device_arch(int dev) {
  hipDeviceProp_t p;
  check(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
  return p.gcnArchName;
}

std::string device_pci_bus_id(int dev) {
  char buf[64] = {0};
  check(hipDeviceGetPCIBusId(buf, sizeof buf, dev), "hipDeviceGetPCIBusId");
  return buf;
}

int device_cu_count(int dev) {
  hipDeviceProp_t p;
  check(hipGetDeviceProperties(&p, dev), "hipGetDeviceProperties");
  return p.multiProcessorCount;
}

// ============================================================================================
// K2a: bf16 MFMA. Operand fragments for v_mfma_f32_32x32x16_bf16 (lane l, r = l&31, h = l>>5):
//   A[row r][k = 8h + j], B[k = 8h + j][col r], j = 0..7;  C/D: col = l&31,
//   row = (reg&3) + 8*(reg>>2) + 4*(l>>5), reg = 0..15   (cdna_hip_programming.md §3)
// ============================================================================================
__device__ __forceinline__ void load_frags(const __bf16* __restrict__ a, const __bf16* __restrict__ b,
                                           int lane, bf16x8* av, bf16x8* bv) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    (*av)[j] = a[r * 16 + 8 * h + j];
    (*bv)[j] = b[(8 * h + j) * 32 + r];
  }
}

__global__ void __launch_bounds__(64) mfma_tile_kernel(const __bf16* __restrict__ a, const __bf16* __restrict__ b,
                                                       float* __restrict__ c, int iters) {
  const int lane = threadIdx.x;
  bf16x8 av, bv;
  load_frags(a, b, lane, &av, &bv);
  f32x16 acc = {};
  for (int i = 0; i < iters; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    c[row * 32 + (lane & 31)] = acc[reg];
  }
}

// Burn: 4 independent accumulators per wave keep the per-SIMD matrix pipe issuing back-to-back
// (32 cycles per 32x32x16 MFMA). Two waves per SIMD (8 per CU) at 2048 blocks of 256 threads.
__global__ void __launch_bounds__(256) mfma_burn_kernel(const __bf16* __restrict__ a, const __bf16* __restrict__ b,
                                                        float* __restrict__ out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 av, bv;
  load_frags(a, b, lane, &av, &bv);
  f32x16 acc0 = {}, acc1 = {}, acc2 = {}, acc3 = {};
  acc1[0] = 1.f;
  acc2[0] = 2.f;
  acc3[0] = 3.f;
  for (int i = 0; i < iters; ++i) {
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc3, 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r] + acc2[r] + acc3[r];
  if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

// ============================================================================================
// K2b: HBM stream. 16 B per lane, non-temporal (streamed once), grid-stride.
// ============================================================================================
__global__ void __launch_bounds__(256) stream_copy_kernel(const i32x4* __restrict__ src, i32x4* __restrict__ dst,
                                                          size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    i32x4 v = __builtin_nontemporal_load(src + i);
    __builtin_nontemporal_store(v, dst + i);
  }
}

// Cache policy of the streamed operands: bit 0 = non-temporal loads, bit 1 = non-temporal stores
// (kStreamNtNt = both, the load generator's choice; the sweep in tools/hbm_sweep.py times all four).
template <int POL>
__device__ __forceinline__ i32x4 ld16(const i32x4* p) {
  if constexpr (POL & 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int POL>
__device__ __forceinline__ void st16(i32x4 v, i32x4* p) {
  if constexpr (POL & 2) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// U independent 16-B loads in flight per lane before the stores (each k-slice of a 256*U-vector
// chunk is one fully coalesced 4 KiB wave-group access); grid-stride over chunks.
template <int U, int POL>
__global__ void __launch_bounds__(256) stream_copy_unrolled_kernel(const i32x4* __restrict__ src,
                                                                   i32x4* __restrict__ dst, size_t n) {
  const size_t chunk = static_cast<size_t>(256) * U;
  for (size_t base = static_cast<size_t>(blockIdx.x) * chunk; base < n; base += static_cast<size_t>(gridDim.x) * chunk) {
    i32x4 v[U];
    if (base + chunk <= n) {
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = ld16<POL>(src + base + k * 256 + threadIdx.x);
#pragma unroll
      for (int k = 0; k < U; ++k) st16<POL>(v[k], dst + base + k * 256 + threadIdx.x);
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const size_t i = base + k * 256 + threadIdx.x;
        if (i < n) st16<POL>(ld16<POL>(src + i), dst + i);
      }
    }
  }
}

// Contiguous-span variant: block b copies [b*span, (b+1)*span) in U-vector chunks, so each CU walks
// one long run of DRAM pages instead of hopping by gridDim*chunk.
template <int U, int POL>
__global__ void __launch_bounds__(256) stream_copy_span_kernel(const i32x4* __restrict__ src, i32x4* __restrict__ dst,
                                                               size_t n, size_t span) {
  const size_t chunk = static_cast<size_t>(256) * U;
  const size_t lo = static_cast<size_t>(blockIdx.x) * span;
  const size_t hi = lo + span < n ? lo + span : n;
  for (size_t base = lo; base < hi; base += chunk) {
    i32x4 v[U];
    if (base + chunk <= hi) {
#pragma unroll
      for (int k = 0; k < U; ++k) v[k] = ld16<POL>(src + base + k * 256 + threadIdx.x);
#pragma unroll
      for (int k = 0; k < U; ++k) st16<POL>(v[k], dst + base + k * 256 + threadIdx.x);
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const size_t i = base + k * 256 + threadIdx.x;
        if (i < hi) st16<POL>(ld16<POL>(src + i), dst + i);
      }
    }
  }
}

__global__ void __launch_bounds__(256) stream_triad_kernel(const f32x4* __restrict__ a,
                                                           const f32x4* __restrict__ b,
                                                           f32x4* __restrict__ c, float s, size_t n4) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 x = __builtin_nontemporal_load(a + i);
    f32x4 y = __builtin_nontemporal_load(b + i);
    f32x4 z;
    z.x = fmaf(s, y.x, x.x);
    z.y = fmaf(s, y.y, x.y);
    z.z = fmaf(s, y.z, x.z);
    z.w = fmaf(s, y.w, x.w);
    __builtin_nontemporal_store(z, c + i);
  }
}

// ============================================================================================
// K1: probe. One wave per workgroup; the stamps are wave-uniform SGPR reads.
//
// Publication to the pinned host ring costs ONE host-memory store per wave plus ONE host flag per
// launch. Each wave writes its 48-byte record as three 16-byte lane stores (one instruction,
// coalesced into one transaction to fine-grained host memory), drains them (vmcnt(0)), then bumps
// a per-slot counter in device memory at agent scope (an L2 atomic: no fabric round trip, no L2
// writeback). The wave that takes the counter to `blocks` re-arms it and publishes the slot with a
// single system-scope store of `blocks` to the host arrival word that the exporter polls.
// The first version did a system-scope release fetch_add on the host word from every wave: 1024
// serialised host atomics each preceded by an L2 writeback (buffer_wbl2), ~1.0 ms per launch on
// MI355X (profiles/r1_probe_publication.md).
// ============================================================================================
__global__ void __launch_bounds__(64) probe_kernel(ProbeRecord* __restrict__ recs, uint32_t* arrivals,
                                                   uint32_t* counter, uint32_t seq, uint32_t spin_ticks,
                                                   uint32_t blocks) {
  probe_body(recs, arrivals, counter, seq, spin_ticks, blocks);  // probe_kernel.h (shared with the HSA path)
}

// ============================================================================================
// host wrappers
// ============================================================================================
void launch_mfma_tile(int dev, const void* a, const void* b, float* c, int iters, void* stream) {
  check(hipSetDevice(dev), "hipSetDevice");
  hipLaunchKernelGGL(mfma_tile_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                     static_cast<const __bf16*>(a), static_cast<const __bf16*>(b), c, iters);
  check(hipGetLastError(), "mfma_tile_kernel");
}

// burn16.hip (own TU, VGPR-form MFMA accumulators)
void launch_mfma_burn16(const __bf16* a, const __bf16* b, float* out, int blocks, int iters, hipStream_t s);

void launch_mfma_burn(int dev, const void* a, const void* b, float* out, int blocks, int iters, void* stream,
                      int shape) {
  check(hipSetDevice(dev), "hipSetDevice");
  auto s = static_cast<hipStream_t>(stream);
  auto pa = static_cast<const __bf16*>(a);
  auto pb = static_cast<const __bf16*>(b);
  if (shape == 32) hipLaunchKernelGGL(mfma_burn_kernel, dim3(blocks), dim3(256), 0, s, pa, pb, out, iters);
  else if (shape == 16) launch_mfma_burn16(pa, pb, out, blocks, iters, s);
  else throw std::invalid_argument("mfma_burn: shape must be 32 (32x32x16) or 16 (16x16x32)");
  check(hipGetLastError(), "mfma_burn_kernel");
}

namespace {
template <int U, int POL>
void copy_launch(hipStream_t s, const i32x4* in, i32x4* out, size_t n16, int blocks, bool span) {
  if (span) {
    const size_t chunk = static_cast<size_t>(256) * U;
    const size_t per = (n16 + blocks - 1) / blocks;
    const size_t sp = (per + chunk - 1) / chunk * chunk;  // whole chunks per block
    hipLaunchKernelGGL((stream_copy_span_kernel<U, POL>), dim3(blocks), dim3(256), 0, s, in, out, n16, sp);
  } else {
    hipLaunchKernelGGL((stream_copy_unrolled_kernel<U, POL>), dim3(blocks), dim3(256), 0, s, in, out, n16);
  }
}
template <int U>
void copy_policy(int policy, hipStream_t s, const i32x4* in, i32x4* out, size_t n16, int blocks, bool span) {
  switch (policy) {
    case 0: copy_launch<U, 3>(s, in, out, n16, blocks, span); break;  // nt loads + nt stores (default)
    case 1: copy_launch<U, 0>(s, in, out, n16, blocks, span); break;  // plain / plain
    case 2: copy_launch<U, 2>(s, in, out, n16, blocks, span); break;  // plain loads, nt stores
    case 3: copy_launch<U, 1>(s, in, out, n16, blocks, span); break;  // nt loads, plain stores
    default: throw std::invalid_argument("stream_copy: policy must be 0..3");
  }
}
}  // namespace

void launch_stream_copy(int dev, const void* src, void* dst, size_t n16, int blocks, void* stream, int unroll,
                        int policy, bool span) {
  check(hipSetDevice(dev), "hipSetDevice");
  if (blocks <= 0) throw std::invalid_argument("stream_copy: blocks must be > 0");
  auto s = static_cast<hipStream_t>(stream);
  auto in = static_cast<const i32x4*>(src);
  auto out = static_cast<i32x4*>(dst);
  switch (unroll) {
    case 1:
      if (policy == 0 && !span) hipLaunchKernelGGL(stream_copy_kernel, dim3(blocks), dim3(256), 0, s, in, out, n16);
      else copy_policy<1>(policy, s, in, out, n16, blocks, span);
      break;
    case 2: copy_policy<2>(policy, s, in, out, n16, blocks, span); break;
    case 4: copy_policy<4>(policy, s, in, out, n16, blocks, span); break;
    case 8: copy_policy<8>(policy, s, in, out, n16, blocks, span); break;
    default: throw std::invalid_argument("stream_copy: unroll must be 1, 2, 4 or 8");
  }
  check(hipGetLastError(), "stream_copy_kernel");
}

void launch_stream_triad(int dev, const float* a, const float* b, float* c, float s, size_t n, int blocks,
                         void* stream) {
  if (n % 4) throw std::invalid_argument("stream_triad: n must be a multiple of 4");
  check(hipSetDevice(dev), "hipSetDevice");
  hipLaunchKernelGGL(stream_triad_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const f32x4*>(a), reinterpret_cast<const f32x4*>(b),
                     reinterpret_cast<f32x4*>(c), s, n / 4);
  check(hipGetLastError(), "stream_triad_kernel");
}

// ---------------------------------------------------------------------------------------------
// LoadGen
// ---------------------------------------------------------------------------------------------
LoadGen::LoadGen(int dev, std::string kind, double duty, size_t hbm_bytes, int mfma_iters)
    : dev_(dev), kind_(std::move(kind)), duty_(std::clamp(duty, 0.01, 1.0)), bytes_(hbm_bytes), iters_(mfma_iters) {
  if (kind_ != "mfma" && kind_ != "hbm" && kind_ != "mixed" && kind_ != "partial" && kind_ != "concurrent")
    throw std::invalid_argument("LoadGen kind must be mfma | hbm | mixed | concurrent | partial");
  bytes_ = std::max<size_t>(bytes_ / 16 * 16, 1 << 20);
}

LoadGen::~LoadGen() { stop(); }

void LoadGen::start() {
  if (running_) return;
  check(hipSetDevice(dev_), "hipSetDevice");
  hipStream_t s;
  check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  stream_ = s;
  if (kind_ == "concurrent") {
    hipStream_t s2;
    check(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking), "hipStreamCreate");
    stream2_ = s2;
  }
  // bf16 operand tile with non-trivial values (keeps the MFMA datapath toggling: realistic power)
  std::vector<uint16_t> h(32 * 16 + 16 * 32);
  for (size_t i = 0; i < h.size(); ++i) {
    float f = std::sin(0.37f * static_cast<float>(i)) * 0.5f;
    uint32_t u;
    memcpy(&u, &f, 4);
    h[i] = static_cast<uint16_t>(u >> 16);
  }
  check(hipMalloc(&a_, h.size() * 2), "hipMalloc");
  b_ = static_cast<char*>(a_) + 32 * 16 * 2;
  check(hipMemcpy(a_, h.data(), h.size() * 2, hipMemcpyHostToDevice), "hipMemcpy");
  check(hipMalloc(reinterpret_cast<void**>(&out_), 4096 * 4 * sizeof(float)), "hipMalloc");
  if (kind_ == "hbm" || kind_ == "mixed" || kind_ == "concurrent") {
    check(hipMalloc(&src_, bytes_), "hipMalloc");
    check(hipMalloc(&dst_, bytes_), "hipMalloc");
    check(hipMemsetAsync(src_, 1, bytes_, s), "hipMemset");
    check(hipStreamSynchronize(s), "hipStreamSynchronize");
  }
  running_ = true;
  t_start_ns_ = mono_ns();
  if (kind_ == "concurrent") {  // two host threads, two streams: both kernels resident at once
    th_ = std::thread([this] { loop(false, true, stream_); });
    th2_ = std::thread([this] { loop(false, false, stream2_); });
  } else {
    th_ = std::thread([this] { loop(kind_ == "mixed", kind_ != "hbm", stream_); });
  }
}

// alternate: flip MFMA / HBM per batch ("mixed"); otherwise `mfma` picks the one kernel kind.
void LoadGen::loop(bool alternate, bool mfma, void* stream) {
  try {
    check(hipSetDevice(dev_), "hipSetDevice");
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipEvent_t e0, e1;
    // GPUMON_LOAD_SYNC=blocking: the batch's completion event is a blocking-sync event, so this host
    // thread sleeps until the GPU interrupt instead of spin-polling for the batch (HIP's default
    // wait): an A/B knob for how a tenant's spinning host thread shows in scrape tails
    // (profiles/r4_scrape_contention.md); default: HIP's default event, as most tenants use.
    const char* sync = getenv("GPUMON_LOAD_SYNC");
    const unsigned ev_flags = sync && !strcmp(sync, "blocking") ? hipEventBlockingSync : hipEventDefault;
    check(hipEventCreateWithFlags(&e0, ev_flags), "hipEventCreate");
    check(hipEventCreateWithFlags(&e1, ev_flags), "hipEventCreate");
    const int cus = device_cu_count(dev_);
    // 8 blocks x 4 waves requested per CU (residency then limited by VGPRs: ~7 waves/SIMD at 68 VGPRs);
    // partial: ~1/4 of the CUs busy; concurrent: 4 waves per SIMD, leaving wave slots for the HBM
    // stream's workgroups (with every slot held by the burn the stream got 0.03 TB/s)
    const int burn_blocks = kind_ == "partial" ? cus / 4 : kind_ == "concurrent" ? cus * 4 : cus * 8;
    // One 16-B vector per lane and one 4 KiB chunk per workgroup, the grid covering the buffer once
    // (no grid-stride loop), nt loads + nt stores: 6.52 TB/s copy on MI355X vs 5.37-5.74 for the
    // earlier 8192 x unroll-4 grid-stride form, 6.20 for PyTorch's elementwise kernel and 4.75 for
    // hipMemcpy D2D in the same interleaved sweep (profiles/r1_hbm_stream.md)
    const size_t n16 = bytes_ / 16;
    const int stream_blocks = static_cast<int>((n16 + 255) / 256);
    bool flip = false;
    while (running_) {
      // one kind per batch so the event time is attributed to exactly one kernel kind
      const bool do_mfma = alternate ? !flip : mfma;
      flip = !flip;
      check(hipEventRecord(e0, s), "hipEventRecord");
      double fl = 0, by = 0;
      for (int k = 0; k < 4; ++k) {
        if (do_mfma && dtype_ != "bf16") {
          fl += launch_mfma_burn_dtype(dev_, dtype_, out_, burn_blocks, iters_, s);
        } else if (do_mfma) {
          launch_mfma_burn(dev_, a_, b_, out_, burn_blocks, iters_, s, shape_);
          fl += static_cast<double>(burn_blocks) * 4 * 4 * iters_ * 32768.0;
        } else {
          launch_stream_copy(dev_, src_, dst_, n16, stream_blocks, s, 1, 0, true);
          by += 2.0 * static_cast<double>(bytes_);
        }
        launches_++;
      }
      check(hipEventRecord(e1, s), "hipEventRecord");
      check(hipEventSynchronize(e1), "hipEventSynchronize");
      float ms = 0;
      check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
      busy_ns_ += static_cast<uint64_t>(ms * 1e6);
      (do_mfma ? mfma_ns_ : hbm_ns_) += static_cast<uint64_t>(ms * 1e6);
      flops_ += static_cast<uint64_t>(fl);
      bytes_moved_ += static_cast<uint64_t>(by);
      if (duty_ < 0.999 && period_s_ > 0) {
        // burst pattern: busy until duty * period into the period, then idle to its end
        const int64_t now = mono_ns();
        const int64_t per = static_cast<int64_t>(period_s_ * 1e9);
        const int64_t phase = (now - t_start_ns_) % per;
        if (phase >= static_cast<int64_t>(duty_ * per)) {
          const int64_t until_ns = now + (per - phase);
          while (running_ && mono_ns() < until_ns) std::this_thread::sleep_for(std::chrono::microseconds(500));
        }
      } else if (duty_ < 0.999) {
        double idle_ms = ms * (1.0 / duty_ - 1.0);
        auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(static_cast<int64_t>(idle_ms * 1e3));
        while (running_ && std::chrono::steady_clock::now() < until)
          std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  } catch (const std::exception& e) {
    err_ = e.what();
    running_ = false;
  }
}

void LoadGen::stop() {
  running_ = false;
  if (th_.joinable()) th_.join();
  if (th2_.joinable()) th2_.join();
  (void)hipSetDevice(dev_);
  for (void** sp : {&stream_, &stream2_}) {
    if (*sp) {
      (void)hipStreamSynchronize(static_cast<hipStream_t>(*sp));
      (void)hipStreamDestroy(static_cast<hipStream_t>(*sp));
      *sp = nullptr;
    }
  }
  if (a_) (void)hipFree(a_);
  if (out_) (void)hipFree(out_);
  if (src_) (void)hipFree(src_);
  if (dst_) (void)hipFree(dst_);
  a_ = b_ = src_ = dst_ = nullptr;
  out_ = nullptr;
}

LoadStats LoadGen::stats() const {
  if (!err_.empty()) throw std::runtime_error("LoadGen failed: " + err_);
  LoadStats s;
  s.launches = launches_;
  s.busy_s = busy_ns_ * 1e-9;
  s.flops = static_cast<double>(flops_.load());
  s.bytes = static_cast<double>(bytes_moved_.load());
  s.mfma_s = mfma_ns_ * 1e-9;
  s.hbm_s = hbm_ns_ * 1e-9;
  s.wall_s = t_start_ns_ ? (mono_ns() - t_start_ns_) * 1e-9 : 0.0;
  return s;
}

// ---------------------------------------------------------------------------------------------
// XgmiLoad: src GPU pushes a buffer into dst GPU memory, back to back, on one src stream.
// ---------------------------------------------------------------------------------------------
XgmiLoad::XgmiLoad(int src, int dst, size_t bytes, std::string method, int blocks)
    : src_(src), dst_(dst), bytes_(std::max<size_t>(bytes / 4096 * 4096, 1 << 20)), method_(std::move(method)),
      blocks_(std::clamp(blocks, 1, 65535)) {
  if (method_ != "kernel" && method_ != "dma") throw std::invalid_argument("XgmiLoad method must be kernel | dma");
  if (src_ == dst_) throw std::invalid_argument("XgmiLoad: src and dst must differ");
  const int n = device_count();
  if (src_ < 0 || dst_ < 0 || src_ >= n || dst_ >= n) throw std::invalid_argument("XgmiLoad: device out of range");
}

XgmiLoad::~XgmiLoad() { stop(); }

void XgmiLoad::start() {
  if (running_) return;
  int can = 0;
  check(hipDeviceCanAccessPeer(&can, src_, dst_), "hipDeviceCanAccessPeer");
  if (!can) throw std::runtime_error("XgmiLoad: device " + std::to_string(src_) + " cannot access peer " +
                                     std::to_string(dst_));
  check(hipSetDevice(dst_), "hipSetDevice");
  check(hipMalloc(&dbuf_, bytes_), "hipMalloc(dst)");
  check(hipSetDevice(src_), "hipSetDevice");
  const hipError_t pe = hipDeviceEnablePeerAccess(dst_, 0);
  if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) check(pe, "hipDeviceEnablePeerAccess");
  (void)hipGetLastError();  // clear a sticky "already enabled"
  hipStream_t s;
  check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  stream_ = s;
  check(hipMalloc(&sbuf_, bytes_), "hipMalloc(src)");
  check(hipMemsetAsync(sbuf_, 3, bytes_, s), "hipMemset");
  check(hipStreamSynchronize(s), "hipStreamSynchronize");
  running_ = true;
  t_start_ns_ = mono_ns();
  th_ = std::thread([this] { loop(); });
}

void XgmiLoad::loop() {
  try {
    check(hipSetDevice(src_), "hipSetDevice");
    hipStream_t s = static_cast<hipStream_t>(stream_);
    hipEvent_t e0, e1;
    check(hipEventCreate(&e0), "hipEventCreate");
    check(hipEventCreate(&e1), "hipEventCreate");
    while (running_) {
      check(hipEventRecord(e0, s), "hipEventRecord");
      for (int k = 0; k < 4; ++k) {
        if (method_ == "dma") check(hipMemcpyPeerAsync(dbuf_, dst_, sbuf_, src_, bytes_, s), "hipMemcpyPeerAsync");
        else launch_stream_copy(src_, sbuf_, dbuf_, bytes_ / 16, blocks_, s, 4, 1, false);  // plain ld / st
      }
      check(hipEventRecord(e1, s), "hipEventRecord");
      check(hipEventSynchronize(e1), "hipEventSynchronize");
      float ms = 0;
      check(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
      busy_ns_ += static_cast<uint64_t>(ms * 1e6);
      copies_ += 4;
      bytes_moved_ += 4 * static_cast<uint64_t>(bytes_);
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  } catch (const std::exception& e) {
    err_ = e.what();
    running_ = false;
  }
}

void XgmiLoad::stop() {
  running_ = false;
  if (th_.joinable()) th_.join();
  if (stream_) {
    (void)hipSetDevice(src_);
    (void)hipStreamSynchronize(static_cast<hipStream_t>(stream_));
    (void)hipStreamDestroy(static_cast<hipStream_t>(stream_));
    stream_ = nullptr;
  }
  if (sbuf_) {
    (void)hipSetDevice(src_);
    (void)hipFree(sbuf_);
  }
  if (dbuf_) {
    (void)hipSetDevice(dst_);
    (void)hipFree(dbuf_);
  }
  sbuf_ = dbuf_ = nullptr;
}

XgmiStats XgmiLoad::stats() const {
  if (!err_.empty()) throw std::runtime_error("XgmiLoad failed: " + err_);
  XgmiStats st;
  st.copies = copies_;
  st.bytes = static_cast<double>(bytes_moved_.load());
  st.busy_s = busy_ns_ * 1e-9;
  st.wall_s = t_start_ns_ ? (mono_ns() - t_start_ns_) * 1e-9 : 0.0;
  return st;
}

// ---------------------------------------------------------------------------------------------
// PcieLoad: the host link's known traffic, the reference for gpu_pcie_bandwidth_bytes_per_second
// (DMA copies from / to pinned host memory: each byte crosses PCIe exactly once)
// ---------------------------------------------------------------------------------------------
PcieLoad::PcieLoad(int dev, size_t bytes, std::string direction, double duty)
    : dev_(dev), bytes_(std::max<size_t>(bytes / 4096 * 4096, 1 << 20)), dir_(std::move(direction)),
      duty_(duty) {
  if (dir_ != "h2d" && dir_ != "d2h" && dir_ != "both") throw std::invalid_argument("PcieLoad direction: h2d | d2h | both");
  if (!(duty_ > 0.0 && duty_ <= 1.0)) throw std::invalid_argument("PcieLoad duty must be in (0, 1]");
  if (dev_ < 0 || dev_ >= device_count()) throw std::invalid_argument("PcieLoad: device out of range");
}

PcieLoad::~PcieLoad() { stop(); }

void PcieLoad::start() {
  if (running_) return;
  check(hipSetDevice(dev_), "hipSetDevice");
  hipStream_t a, b;
  check(hipStreamCreateWithFlags(&a, hipStreamNonBlocking), "hipStreamCreate");
  up_ = a;
  check(hipStreamCreateWithFlags(&b, hipStreamNonBlocking), "hipStreamCreate");
  down_ = b;
  check(hipHostMalloc(&host_src_, bytes_, hipHostMallocDefault), "hipHostMalloc(src)");
  check(hipHostMalloc(&host_dst_, bytes_, hipHostMallocDefault), "hipHostMalloc(dst)");
  memset(host_src_, 5, bytes_);
  check(hipMalloc(&dev_src_, bytes_), "hipMalloc(src)");
  check(hipMalloc(&dev_dst_, bytes_), "hipMalloc(dst)");
  check(hipMemsetAsync(dev_src_, 7, bytes_, a), "hipMemset");
  check(hipStreamSynchronize(a), "hipStreamSynchronize");
  running_ = true;
  t_start_ns_ = mono_ns();
  th_ = std::thread([this] { loop(); });
}

void PcieLoad::loop() {
  try {
    check(hipSetDevice(dev_), "hipSetDevice");
    hipStream_t a = static_cast<hipStream_t>(up_), b = static_cast<hipStream_t>(down_);
    const bool up = dir_ != "d2h", down = dir_ != "h2d";
    hipEvent_t e[4];
    for (auto& x : e) check(hipEventCreate(&x), "hipEventCreate");
    while (running_) {
      const int64_t t0 = mono_ns();
      if (up) check(hipEventRecord(e[0], a), "hipEventRecord");
      if (down) check(hipEventRecord(e[2], b), "hipEventRecord");
      for (int k = 0; k < 2; ++k) {
        if (up) check(hipMemcpyAsync(dev_dst_, host_src_, bytes_, hipMemcpyHostToDevice, a), "hipMemcpyAsync(h2d)");
        if (down) check(hipMemcpyAsync(host_dst_, dev_src_, bytes_, hipMemcpyDeviceToHost, b), "hipMemcpyAsync(d2h)");
      }
      if (up) check(hipEventRecord(e[1], a), "hipEventRecord");
      if (down) check(hipEventRecord(e[3], b), "hipEventRecord");
      float ms_up = 0, ms_down = 0;
      if (up) {
        check(hipEventSynchronize(e[1]), "hipEventSynchronize");
        check(hipEventElapsedTime(&ms_up, e[0], e[1]), "hipEventElapsedTime");
        h2d_ += 2 * static_cast<uint64_t>(bytes_);
      }
      if (down) {
        check(hipEventSynchronize(e[3]), "hipEventSynchronize");
        check(hipEventElapsedTime(&ms_down, e[2], e[3]), "hipEventElapsedTime");
        d2h_ += 2 * static_cast<uint64_t>(bytes_);
      }
      busy_ns_ += static_cast<uint64_t>(std::max(ms_up, ms_down) * 1e6);
      copies_ += (up ? 2 : 0) + (down ? 2 : 0);
      if (duty_ < 1.0) {
        // idle for (1 - duty) / duty of the batch just run, in <= 50 ms slices so stop() is prompt
        int64_t left = static_cast<int64_t>((mono_ns() - t0) * (1.0 / duty_ - 1.0));
        while (running_ && left > 0) {
          const int64_t s = std::min<int64_t>(left, 50'000'000);
          std::this_thread::sleep_for(std::chrono::nanoseconds(s));
          left -= s;
        }
      }
    }
    for (auto& x : e) (void)hipEventDestroy(x);
  } catch (const std::exception& ex) {
    err_ = ex.what();
    running_ = false;
  }
}

void PcieLoad::stop() {
  running_ = false;
  if (th_.joinable()) th_.join();
  (void)hipSetDevice(dev_);
  for (void** s : {&up_, &down_})
    if (*s) {
      (void)hipStreamSynchronize(static_cast<hipStream_t>(*s));
      (void)hipStreamDestroy(static_cast<hipStream_t>(*s));
      *s = nullptr;
    }
  for (void** p : {&host_src_, &host_dst_})
    if (*p) {
      (void)hipHostFree(*p);
      *p = nullptr;
    }
  for (void** p : {&dev_src_, &dev_dst_})
    if (*p) {
      (void)hipFree(*p);
      *p = nullptr;
    }
}

PcieStats PcieLoad::stats() const {
  if (!err_.empty()) throw std::runtime_error("PcieLoad failed: " + err_);
  PcieStats st;
  st.copies = copies_;
  st.h2d_bytes = static_cast<double>(h2d_.load());
  st.d2h_bytes = static_cast<double>(d2h_.load());
  st.busy_s = busy_ns_ * 1e-9;
  st.wall_s = t_start_ns_ ? (mono_ns() - t_start_ns_) * 1e-9 : 0.0;
  return st;
}

// ---------------------------------------------------------------------------------------------
// Probe
// ---------------------------------------------------------------------------------------------
Probe::Probe(int dev, int blocks, int slots, int spin_ticks)
    : dev_(dev), blocks_(std::max(1, blocks)), slots_(std::max(1, slots)), spin_(std::max(1, spin_ticks)) {
  check(hipSetDevice(dev_), "hipSetDevice");
  // Every HIP stream is a hardware queue, and on MI355X each queue pins a ~173 MB host context-save
  // area (profiles/r2_footprint.md). GPUMON_PROBE_STREAM=null runs the probe on the device's null
  // stream instead of a stream of its own (the helper issues nothing else through HIP).
  hipStream_t s = nullptr;
  const char* mode = getenv("GPUMON_PROBE_STREAM");
  if (!(mode && !strcmp(mode, "null"))) check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  stream_ = s;
  const size_t rb = sizeof(ProbeRecord) * static_cast<size_t>(blocks_) * slots_;
  check(hipHostMalloc(reinterpret_cast<void**>(&ring_), rb, hipHostMallocMapped | hipHostMallocCoherent),
        "hipHostMalloc(ring)");
  check(hipHostMalloc(reinterpret_cast<void**>(&arrivals_), sizeof(uint32_t) * slots_,
                      hipHostMallocMapped | hipHostMallocCoherent),
        "hipHostMalloc(arrivals)");
  memset(ring_, 0, rb);
  memset(arrivals_, 0, sizeof(uint32_t) * slots_);
  check(hipHostGetDevicePointer(reinterpret_cast<void**>(&ring_dev_), ring_, 0), "hipHostGetDevicePointer");
  check(hipHostGetDevicePointer(reinterpret_cast<void**>(&arrivals_dev_), arrivals_, 0), "hipHostGetDevicePointer");
  check(hipMalloc(reinterpret_cast<void**>(&counters_dev_), sizeof(uint32_t) * slots_), "hipMalloc(counters)");
  check(hipMemsetAsync(counters_dev_, 0, sizeof(uint32_t) * slots_, s), "hipMemset(counters)");
  check(hipStreamSynchronize(s), "hipStreamSynchronize");
  slot_seq_.assign(slots_, 0);
  slot_launch_ns_.assign(slots_, 0);
}

Probe::~Probe() {
  (void)hipSetDevice(dev_);
  if (stream_) {
    (void)hipStreamSynchronize(static_cast<hipStream_t>(stream_));
    (void)hipStreamDestroy(static_cast<hipStream_t>(stream_));
  }
  if (ring_) (void)hipHostFree(ring_);
  if (arrivals_) (void)hipHostFree(arrivals_);
  if (counters_dev_) (void)hipFree(counters_dev_);
}

int Probe::launch() {
  const int slot = next_;
  // A slot is reusable only when its previous launch fully arrived.
  if (slot_seq_[slot] != 0 && __atomic_load_n(&arrivals_[slot], __ATOMIC_ACQUIRE) < static_cast<uint32_t>(blocks_))
    return -1;
  next_ = (next_ + 1) % slots_;
  const uint32_t seq = ++seq_;
  __atomic_store_n(&arrivals_[slot], 0u, __ATOMIC_RELEASE);
  slot_seq_[slot] = seq;
  check(hipSetDevice(dev_), "hipSetDevice");
  slot_launch_ns_[slot] = mono_ns();
  hipLaunchKernelGGL(probe_kernel, dim3(blocks_), dim3(64), 0, static_cast<hipStream_t>(stream_),
                     ring_dev_ + static_cast<size_t>(slot) * blocks_, arrivals_dev_ + slot, counters_dev_ + slot, seq,
                     static_cast<uint32_t>(spin_), static_cast<uint32_t>(blocks_));
  check(hipGetLastError(), "probe_kernel");
  return slot;
}

bool Probe::poll(int slot, ProbeResult* out) {
  if (slot < 0 || slot >= slots_) return false;
  const uint32_t arrived = __atomic_load_n(&arrivals_[slot], __ATOMIC_ACQUIRE);
  out->seq = slot_seq_[slot];
  out->blocks = blocks_;
  out->arrived = static_cast<int>(arrived);
  out->host_launch_ns = slot_launch_ns_[slot];
  if (arrived < static_cast<uint32_t>(blocks_)) {
    out->complete = false;
    return false;
  }
  out->complete = true;
  out->host_done_ns = mono_ns();
  probe_collect(ring_ + static_cast<size_t>(slot) * blocks_, blocks_, out);
  return true;
}

bool Probe::wait(int slot, double timeout_s, ProbeResult* out) {
  const int64_t deadline = mono_ns() + static_cast<int64_t>(timeout_s * 1e9);
  while (!poll(slot, out)) {
    if (mono_ns() > deadline) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  return true;
}

}  // namespace gpumon_hip
