// Host side of the K1 probe, shared by the HIP launch path (gpumon_hip::Probe, kernels.hip) and the
// raw-HSA one (csrc/plugins/probe_hsa.cpp): what a launch's records say once its arrival flag has
// reached `blocks`. No GPU runtime here: the records are plain host memory.
#pragma once

#include <algorithm>
#include <cstdint>
#include <map>
#include <set>
#include <thread>
#include <tuple>
#include <vector>

#include "kernels.h"

namespace gpumon_hip {

struct ProbeResult {
  bool complete = false;
  uint32_t seq = 0;
  int blocks = 0;
  int arrived = 0;
  int64_t host_launch_ns = 0;   // CLOCK_MONOTONIC before the launch call
  int64_t host_done_ns = 0;     // when the host observed the last arrival
  uint64_t gpu_span_ticks = 0;  // max(t1) - min(t0), 100 MHz ticks
  uint64_t gpu_first_start = 0; // min(t0) in ticks
  std::vector<int> xcc_blocks;  // blocks seen per XCC id (index 0..15)
  std::vector<double> xcc_clock_mhz;  // mean effective shader clock per XCC (0 if none)
  int unique_cus = 0;
  std::vector<double> xcc_wave_slot;  // mean lowest HW_ID.WAVE_ID per SIMD, per XCC (resident-wave pressure)
  double wave_slot_mean = 0;          // the same over every SIMD seen
  int stale_records = 0;        // records whose seq never matched after the flag (should be 0)
  std::vector<ProbeRecord> records;
};

// `r` = the slot's `blocks` records in the pinned ring; out->seq = the launch's sequence number.
inline void probe_collect(const ProbeRecord* r, int blocks, ProbeResult* out) {
  // The flag is written after every wave drained its record stores; a record still in flight on
  // another fabric path would show the previous seq. Re-read those briefly (bounded) and count what
  // never landed.
  std::vector<int> late;
  for (int b = 0; b < blocks; ++b)
    if (__atomic_load_n(&r[b].seq, __ATOMIC_ACQUIRE) != out->seq) late.push_back(b);
  for (int spin = 0; !late.empty() && spin < 1000; ++spin) {
    std::this_thread::yield();
    late.erase(std::remove_if(late.begin(), late.end(),
                              [&](int b) { return __atomic_load_n(&r[b].seq, __ATOMIC_ACQUIRE) == out->seq; }),
               late.end());
  }
  out->stale_records = static_cast<int>(late.size());
  out->records.assign(r, r + blocks);
  out->xcc_blocks.assign(16, 0);
  std::vector<double> clk_sum(16, 0.0);
  uint64_t tmin = ~0ull, tmax = 0;
  std::set<std::tuple<uint32_t, uint32_t>> cus;
  for (const auto& x : out->records) {
    if (x.seq != out->seq) continue;  // torn / stale record (should not happen after the counter)
    const uint32_t xc = x.xcc_id & 0xF;
    out->xcc_blocks[xc]++;
    const uint64_t dt = x.t1_real - x.t0_real;
    if (dt) clk_sum[xc] += static_cast<double>(x.c1 - x.c0) / static_cast<double>(dt) * 100.0;  // MHz
    tmin = std::min(tmin, x.t0_real);
    tmax = std::max(tmax, x.t1_real);
    // CU identity inside an XCC: HW_ID bits [15:8] = cu_id | sh_id | se_id
    cus.insert({xc, (x.hw_id >> 8) & 0xFF});
  }
  // Resident-wave pressure: the SPI hands a new wave the lowest free slot of its SIMD, so the lowest
  // WAVE_ID a probe wave got on a SIMD counts the slots other work held there at launch.
  std::map<uint32_t, uint32_t> simd_min;  // (xcc, se, sh, cu, simd) -> lowest wave slot
  for (const auto& x : out->records) {
    if (x.seq != out->seq) continue;
    const uint32_t key = ((x.xcc_id & 0xF) << 16) | (((x.hw_id >> 8) & 0xFF) << 2) | ((x.hw_id >> 4) & 0x3);
    const uint32_t slot = x.hw_id & 0xF;
    auto it = simd_min.find(key);
    if (it == simd_min.end()) simd_min.emplace(key, slot);
    else it->second = std::min(it->second, slot);
  }
  std::vector<double> ws_sum(16, 0.0), ws_n(16, 0.0);
  double all = 0;
  for (const auto& kv : simd_min) {
    ws_sum[kv.first >> 16] += kv.second;
    ws_n[kv.first >> 16] += 1;
    all += kv.second;
  }
  out->xcc_wave_slot.assign(16, 0.0);
  for (int k = 0; k < 16; ++k)
    if (ws_n[k] > 0) out->xcc_wave_slot[k] = ws_sum[k] / ws_n[k];
  out->wave_slot_mean = simd_min.empty() ? 0.0 : all / simd_min.size();
  out->xcc_clock_mhz.assign(16, 0.0);
  for (int k = 0; k < 16; ++k)
    if (out->xcc_blocks[k]) out->xcc_clock_mhz[k] = clk_sum[k] / out->xcc_blocks[k];
  out->gpu_first_start = tmin;
  out->gpu_span_ticks = tmax > tmin ? tmax - tmin : 0;
  out->unique_cus = static_cast<int>(cus.size());
}

}  // namespace gpumon_hip
