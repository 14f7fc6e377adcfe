// Host-side API over the gfx950 kernels (implemented in kernels.hip, bound in hip_module.cpp).
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

#include "kernels.h"
#include "probe_collect.h"

namespace gpumon_hip {

void check(int err, const char* what);  // throws std::runtime_error on a HIP error

int device_count();
std::string device_arch(int dev);
int device_cu_count(int dev);
// PCI address of a HIP ordinal ("0000:75:00.0", hipDeviceGetPCIBusId): how a process that sees a
// subset of the node (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES) names its GPUs to the exporter,
// whose hip_id is node-wide (gpumon/parallel/devmap.py).
std::string device_pci_bus_id(int dev);

// --- numerics-testable launches on caller-provided device pointers / streams -------------------
// C[32x32] (fp32, row-major) = iters * A[32x16] @ B[16x32] (bf16, row-major), one wave.
void launch_mfma_tile(int dev, const void* a, const void* b, float* c, int iters, void* stream);
// Burn: `blocks` x 256 threads; each wave runs iters x 4 MFMAs; wave sums go to out[blocks*4].
// shape 32: v_mfma_f32_32x32x16_bf16 x4 accumulators; 16: v_mfma_f32_16x16x32_bf16 x8 (same FLOP/iter)
void launch_mfma_burn(int dev, const void* a, const void* b, float* out, int blocks, int iters, void* stream,
                      int shape = 32);
// Burns of the other matrix paths (burn_dtypes.hip): dtype f16 | fp8 | f32 | f64 | i8 | mxfp8 | mxfp4.
// Same geometry as the bf16 burn (256-thread workgroups, 8 chains/wave); returns FLOP per launch.
double launch_mfma_burn_dtype(int dev, const std::string& dtype, float* out, int blocks, int iters, void* stream);
// dst = src (n16 = number of 16-byte vectors)
// policy: 0 nt loads + nt stores, 1 plain, 2 plain loads + nt stores, 3 nt loads + plain stores;
// span: each block copies one contiguous range instead of grid-striding
void launch_stream_copy(int dev, const void* src, void* dst, size_t n16, int blocks, void* stream, int unroll = 4,
                        int policy = 0, bool span = false);
// c = a + s * b  (fp32, n elements, n % 4 == 0)
void launch_stream_triad(int dev, const float* a, const float* b, float* c, float s, size_t n, int blocks,
                         void* stream);

// --- background synthetic load ----------------------------------------------------------------
struct LoadStats {
  uint64_t launches = 0;
  double busy_s = 0;        // GPU time measured with events
  double flops = 0;         // MFMA FLOP issued
  double bytes = 0;         // HBM bytes moved (read + write)
  double mfma_s = 0;        // GPU time of MFMA batches
  double hbm_s = 0;         // GPU time of HBM-stream batches
  double wall_s = 0;        // wall time since start() (rates over wall time = flops / wall_s)
};

class LoadGen {
 public:
  // kind: "mfma" | "hbm" | "mixed" (alternating MFMA / HBM batches on one stream) | "concurrent"
  // (MFMA burn and HBM stream on two streams at the same time: both pipes loaded at once, the
  // power/thermal worst case) | "partial" (a quarter of the CUs burning);
  // duty in (0, 1]: fraction of wall time the GPU is kept busy
  LoadGen(int dev, std::string kind, double duty, size_t hbm_bytes, int mfma_iters);
  ~LoadGen();
  void start();
  void stop();
  LoadStats stats() const;
  bool running() const { return running_; }
  void set_mfma_shape(int shape) { shape_ = shape; }  // 32 or 16 (launch_mfma_burn); before start()
  // bf16 (the shape above) or a launch_mfma_burn_dtype path: f16 fp8 f32 f64 i8 mxfp8 mxfp4; before start()
  void set_mfma_dtype(std::string dtype) { dtype_ = std::move(dtype); }
  int mfma_shape() const { return shape_; }
  // > 0: duty cycle as long bursts, duty * period_s busy then (1 - duty) * period_s idle (step /
  // communication phases), instead of an idle gap after every batch; before start()
  void set_period(double period_s) { period_s_ = period_s; }

 private:
  void loop(bool alternate, bool mfma, void* stream);
  int dev_;
  std::string kind_;
  double duty_;
  size_t bytes_;
  int iters_;
  int shape_ = 32;
  double period_s_ = 0;
  std::string dtype_ = "bf16";
  void* stream_ = nullptr;
  void* stream2_ = nullptr;  // "concurrent": the HBM stream's own HIP stream
  void* a_ = nullptr;
  void* b_ = nullptr;
  float* out_ = nullptr;
  void* src_ = nullptr;
  void* dst_ = nullptr;
  std::thread th_, th2_;
  std::atomic<bool> running_{false};
  int64_t t_start_ns_ = 0;
  mutable std::atomic<uint64_t> launches_{0};
  std::atomic<uint64_t> busy_ns_{0};
  std::atomic<uint64_t> flops_{0};
  std::atomic<uint64_t> bytes_moved_{0};
  std::atomic<uint64_t> mfma_ns_{0}, hbm_ns_{0};
  std::string err_;
};

// --- xGMI load: one GPU pushes to one peer (drives exactly the link between them) ---------------
struct XgmiStats {
  uint64_t copies = 0;
  double bytes = 0;    // bytes that crossed the link
  double busy_s = 0;   // event-timed GPU time of the copies
  double wall_s = 0;   // since start()
};

class XgmiLoad {
 public:
  // method "kernel": a copy kernel on `src` reads local HBM and stores into `dst`'s memory through
  //                  the peer mapping (the store stream crosses the src->dst xGMI link);
  //        "dma":    hipMemcpyPeerAsync on a src-device stream.
  XgmiLoad(int src, int dst, size_t bytes, std::string method, int blocks);
  ~XgmiLoad();
  void start();
  void stop();
  XgmiStats stats() const;
  bool running() const { return running_; }

 private:
  void loop();
  int src_, dst_;
  size_t bytes_;
  std::string method_;
  int blocks_;
  void* stream_ = nullptr;
  void* sbuf_ = nullptr;  // on src
  void* dbuf_ = nullptr;  // on dst
  std::thread th_;
  std::atomic<bool> running_{false};
  int64_t t_start_ns_ = 0;
  std::atomic<uint64_t> copies_{0}, bytes_moved_{0}, busy_ns_{0};
  std::string err_;
};

// --- PCIe load: pinned host <-> device copies (drives the device's PCIe link) ----------------------
struct PcieStats {
  uint64_t copies = 0;
  double h2d_bytes = 0, d2h_bytes = 0;  // bytes that crossed the link, per direction
  double busy_s = 0;                    // event-timed GPU time of the copy batches
  double wall_s = 0;                    // since start()
};

class PcieLoad {
 public:
  // direction "h2d" | "d2h" | "both" (the two directions on two streams at once); duty in (0, 1]:
  // share of wall time spent copying (idle gaps sized from each batch's event-timed length)
  PcieLoad(int dev, size_t bytes, std::string direction, double duty);
  ~PcieLoad();
  void start();
  void stop();
  PcieStats stats() const;
  bool running() const { return running_; }

 private:
  void loop();
  int dev_;
  size_t bytes_;
  std::string dir_;
  double duty_;
  void* up_ = nullptr;    // h2d stream
  void* down_ = nullptr;  // d2h stream
  void* host_src_ = nullptr;  // pinned
  void* host_dst_ = nullptr;  // pinned
  void* dev_src_ = nullptr;
  void* dev_dst_ = nullptr;
  std::thread th_;
  std::atomic<bool> running_{false};
  int64_t t_start_ns_ = 0;
  std::atomic<uint64_t> copies_{0}, h2d_{0}, d2h_{0}, busy_ns_{0};
  std::string err_;
};

// --- K1 probe: pinned ring buffer ----------------------------------------------------------------
class Probe {
 public:
  Probe(int dev, int blocks, int slots, int spin_ticks);
  ~Probe();
  int launch();                              // returns slot; non-blocking
  bool poll(int slot, ProbeResult* out);     // true when complete (no device sync)
  bool wait(int slot, double timeout_s, ProbeResult* out);
  int blocks() const { return blocks_; }

 private:
  int dev_, blocks_, slots_, spin_;
  void* stream_ = nullptr;
  ProbeRecord* ring_ = nullptr;         // host pinned, device mapped
  uint32_t* arrivals_ = nullptr;        // host pinned, one counter per slot
  ProbeRecord* ring_dev_ = nullptr;
  uint32_t* arrivals_dev_ = nullptr;
  uint32_t* counters_dev_ = nullptr;   // device memory, one arrival counter per slot (self re-arming)
  std::vector<uint32_t> slot_seq_;
  std::vector<int64_t> slot_launch_ns_;
  uint32_t seq_ = 0;
  int next_ = 0;
};

}  // namespace gpumon_hip
