// Can a shader read what the SQ is doing? gfx940+ exposes four read-only hardware registers to
// s_getreg_b32 -- HW_REG_SQ_PERF_SNAPSHOT_DATA / _DATA1 / _PC_LO / _PC_HI -- the state the SQ
// latches for stochastic (trap-based) PC sampling. If they are live without a profiler arming
// them, an in-kernel reader could sample other waves' PCs and instruction types on its CU: the
// "SQ perf counters read by a microkernel" of the BASELINE north star, which the probe design
// (docs/architecture.md, "PMC") ruled out for the SQ/GRBM *counter* registers.
//
// Experiment (bounded: every loop has a fixed trip count; no device-wide waits):
//   1. reader alone: 256 one-wave workgroups, each reads the four registers 256 times with a
//      short s_sleep between reads, stores them (vector stores) to device memory;
//   2. the same reader on a second stream while a VALU burn (known PC range) occupies every CU.
// The host reports how many reads were non-zero, how many distinct values appeared, and whether
// any sampled PC falls in the burn's or the reader's own code.
//
//   hipcc --offload-arch=gfx950 -O2 tools/perf_snapshot_probe.hip -o build/perf_snapshot_probe
//   build/perf_snapshot_probe  > gpurun_out/snapshot.json
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                           \
    }                                                                                         \
  } while (0)

constexpr int kReaders = 256;
constexpr int kReads = 256;

struct Snap {
  uint32_t data, data1, pc_lo, pc_hi;
};

__global__ void __launch_bounds__(64) snapshot_reader(Snap* __restrict__ out, uint64_t* __restrict__ own_pc) {
  uint64_t pc;
  asm volatile("s_getpc_b64 %0" : "=s"(pc));
  if (blockIdx.x == 0 && threadIdx.x == 0) *own_pc = pc;
  for (int i = 0; i < kReads; ++i) {
    uint32_t d, d1, lo, hi;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_SQ_PERF_SNAPSHOT_DATA)" : "=s"(d));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_SQ_PERF_SNAPSHOT_DATA1)" : "=s"(d1));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_SQ_PERF_SNAPSHOT_PC_LO)" : "=s"(lo));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_SQ_PERF_SNAPSHOT_PC_HI)" : "=s"(hi));
    if (threadIdx.x == 0) out[blockIdx.x * kReads + i] = Snap{d, d1, lo, hi};
    __builtin_amdgcn_s_sleep(8);
  }
}

__global__ void __launch_bounds__(256) valu_burn(float* __restrict__ sink, uint64_t* __restrict__ own_pc, int iters) {
  uint64_t pc;
  asm volatile("s_getpc_b64 %0" : "=s"(pc));
  if (blockIdx.x == 0 && threadIdx.x == 0) *own_pc = pc;
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.9999f, d = blockIdx.x * 1e-4f;
  for (int i = 0; i < iters; ++i) {
    a = fmaf(a, b, c);
    d = fmaf(d, c, b);
    b = fmaf(b, c, a * 1e-7f);
    c = fmaf(c, b, d * 1e-7f);
  }
  if (a + b + c + d == 12345.0f) sink[blockIdx.x] = a;  // keep the chain alive
}

static void report(const char* name, const std::vector<Snap>& s, uint64_t reader_pc, uint64_t burn_pc, bool last) {
  size_t nz = 0, in_burn = 0, in_reader = 0;
  std::set<uint64_t> distinct, pcs;
  for (const Snap& x : s) {
    if (x.data | x.data1 | x.pc_lo | x.pc_hi) ++nz;
    distinct.insert((uint64_t(x.data) << 32) | x.data1);
    const uint64_t pc = (uint64_t(x.pc_hi) << 32) | x.pc_lo;
    pcs.insert(pc);
    if (burn_pc && pc >= burn_pc - 4096 && pc < burn_pc + 4096) ++in_burn;
    if (reader_pc && pc >= reader_pc - 4096 && pc < reader_pc + 4096) ++in_reader;
  }
  std::printf("  \"%s\": {\"reads\": %zu, \"nonzero\": %zu, \"distinct_data\": %zu, \"distinct_pc\": %zu, "
              "\"pc_in_burn\": %zu, \"pc_in_reader\": %zu, \"first\": [",
              name, s.size(), nz, distinct.size(), pcs.size(), in_burn, in_reader);
  int shown = 0;
  for (size_t i = 0; i < s.size() && shown < 8; ++i) {
    if (!(s[i].data | s[i].data1 | s[i].pc_lo | s[i].pc_hi) && i > 0) continue;
    std::printf("%s[\"0x%08x\", \"0x%08x\", \"0x%08x%08x\"]", shown ? ", " : "", s[i].data, s[i].data1, s[i].pc_hi,
                s[i].pc_lo);
    ++shown;
  }
  std::printf("]}%s\n", last ? "" : ",");
}

int main(int argc, char** argv) {
  const int burn_iters = argc > 1 ? std::atoi(argv[1]) : (1 << 21);
  CHECK(hipSetDevice(0));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  Snap* d_out;
  uint64_t *d_pc, h_pc[2] = {0, 0};
  float* sink;
  const size_t n = size_t(kReaders) * kReads;
  CHECK(hipMalloc(&d_out, n * sizeof(Snap)));
  CHECK(hipMalloc(&d_pc, 2 * sizeof(uint64_t)));
  CHECK(hipMalloc(&sink, 4096 * sizeof(float)));
  CHECK(hipMemset(d_pc, 0, 2 * sizeof(uint64_t)));
  std::vector<Snap> idle(n), loaded(n);

  // 1. reader alone
  CHECK(hipMemsetAsync(d_out, 0, n * sizeof(Snap), s1));
  hipLaunchKernelGGL(snapshot_reader, dim3(kReaders), dim3(64), 0, s1, d_out, d_pc);
  CHECK(hipGetLastError());
  CHECK(hipStreamSynchronize(s1));
  CHECK(hipMemcpy(idle.data(), d_out, n * sizeof(Snap), hipMemcpyDeviceToHost));

  // 2. reader next to a VALU burn: 1024 x 256 threads = 4 waves per SIMD on 256 CUs, leaving slots
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipMemsetAsync(d_out, 0, n * sizeof(Snap), s1));
  CHECK(hipStreamSynchronize(s1));
  CHECK(hipEventRecord(e0, s2));
  hipLaunchKernelGGL(valu_burn, dim3(1024), dim3(256), 0, s2, sink, d_pc + 1, burn_iters);
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e1, s2));
  hipLaunchKernelGGL(snapshot_reader, dim3(kReaders), dim3(64), 0, s1, d_out, d_pc);
  CHECK(hipGetLastError());
  CHECK(hipStreamSynchronize(s1));
  const bool burn_running_at_reader_end = hipEventQuery(e1) == hipErrorNotReady;
  CHECK(hipStreamSynchronize(s2));
  float burn_ms = 0;
  CHECK(hipEventElapsedTime(&burn_ms, e0, e1));
  CHECK(hipMemcpy(loaded.data(), d_out, n * sizeof(Snap), hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h_pc, d_pc, sizeof(h_pc), hipMemcpyDeviceToHost));

  std::printf("{\n  \"reader_pc\": \"0x%llx\", \"burn_pc\": \"0x%llx\", \"burn_ms\": %.2f, "
              "\"burn_running_when_reader_done\": %s,\n",
              (unsigned long long)h_pc[0], (unsigned long long)h_pc[1], burn_ms,
              burn_running_at_reader_end ? "true" : "false");
  report("idle", idle, h_pc[0], h_pc[1], false);
  report("under_valu_burn", loaded, h_pc[0], h_pc[1], true);
  std::printf("}\n");
  CHECK(hipFree(d_out));
  CHECK(hipFree(d_pc));
  CHECK(hipFree(sink));
  return 0;
}
