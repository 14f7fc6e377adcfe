// Accumulator -> rate conversion (energy, throttle residencies, per-XCD busy, xGMI bytes).
//
// The reference computes no rates at all: it re-reads instantaneous nvidia-smi values every
// ~13-19 s (/root/reference/gpu.py:104-109). MI355X firmware exposes monotone
// accumulators in the gpu_metrics table; rates over the sampling interval are both more accurate
// than instantaneous values and free (no extra calls). First tick after start/reset: no rate.
#pragma once

#include "sample.h"

namespace gpumon {

// gfx_activity_acc / gfx_busy_acc accumulate the instantaneous busy % once per
// accumulation_counter tick, so avg% = d(acc) / d(accumulation_counter) (MI355X: ~3.45 % lifetime
// average read on an idle box = 724166309 / 209992046). `activity_acc_scale` is a correction hook.
// Calibrated on MI355X (see tests/gpu/test_amdsmi_backend.py); overridable for other firmware.
struct RateConfig {
  double activity_acc_scale = 1.0;   // avg% = d(acc) / d(accumulation_counter) * scale
  double xgmi_kb_bytes = 1024.0;     // bytes per xGMI "KB" accumulator unit
  // Bytes/s per unit of pcie_bandwidth_inst / per accumulation tick of pcie_bandwidth_acc. The
  // kernel header calls them GB/s; on MI355X (gpu_metrics v1.8) an idle GPU reads 18-21 and a
  // 57.4 GB/s pinned host->device copy 558481: 102400 B/s per unit (100 KiB/s) puts h2d within
  // 0.4 %, a 50 % duty h2d within 0.2 %, d2h 6 % under and both directions 2.6 % under the copies'
  // host-clocked rates (tools/pcie_probe.py, profiles/r6_pcie_bandwidth.md).
  double pcie_bw_unit_bytes = 102400.0;
};

// Unsigned delta that tolerates a 32-bit firmware wrap when `bits32` is set; returns false on a
// backwards step (device reset / driver reload) so the caller skips the rate for this tick.
bool acc_delta(uint64_t prev, uint64_t cur, bool bits32, uint64_t* out);

void compute_rates(const DeviceSample& prev, const DeviceSample& cur, const RateConfig& cfg,
                   DeviceRates* out);

}  // namespace gpumon
