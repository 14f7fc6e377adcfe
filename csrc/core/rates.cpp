#include "rates.h"

#include <algorithm>

namespace gpumon {

bool acc_delta(uint64_t prev, uint64_t cur, bool bits32, uint64_t* out) {
  if (bits32) {
    *out = (static_cast<uint32_t>(cur) - static_cast<uint32_t>(prev)) & 0xFFFFFFFFull;
    // A 32-bit wrap is legitimate; a huge jump is not (treat > 2^31 as a reset).
    return *out < (1ull << 31);
  }
  if (cur < prev) return false;
  *out = cur - prev;
  return true;
}

void compute_rates(const DeviceSample& prev, const DeviceSample& cur, const RateConfig& cfg,
                   DeviceRates* out) {
  *out = DeviceRates{};
  if (!prev.ok || !cur.ok || !prev.acc.valid || !cur.acc.valid) return;
  const Accumulators& a = prev.acc;
  const Accumulators& b = cur.acc;
  // Time base. The accumulators move only when the firmware rewrites its table (every 20 ms on
  // MI355X, profiles/r3_capacity.md), while system_clock_counter is stamped by the driver at each
  // read: a read-time dt is off by up to one firmware period per interval (+-2 % at 1 Hz, +-20 %
  // at 10 Hz). The firmware's own timestamp (10 ns units) spans exactly the accumulated window;
  // it is used when it advanced and agrees with the read-time dt to within a factor of two.
  double dt_read = 0;
  if (a.system_clock_ns && b.system_clock_ns && b.system_clock_ns > a.system_clock_ns)
    dt_read = (b.system_clock_ns - a.system_clock_ns) * 1e-9;
  else if (cur.host_mono_ns > prev.host_mono_ns)
    dt_read = (cur.host_mono_ns - prev.host_mono_ns) * 1e-9;
  double dt = dt_read;
  if (a.firmware_ts && b.firmware_ts > a.firmware_ts) {
    const double dt_fw = (b.firmware_ts - a.firmware_ts) * 1e-8;
    if (dt_read <= 0 || (dt_fw >= 0.5 * dt_read - 0.05 && dt_fw <= 2.0 * dt_read + 0.05)) dt = dt_fw;
  }
  if (dt <= 0) return;
  out->valid = true;
  out->dt_s = dt;
  uint64_t d = 0;
  if (b.energy && acc_delta(a.energy, b.energy, false, &d))
    out->power_from_energy_w = d * b.energy_resolution_uj * 1e-6 / dt;
  uint64_t dacc = 0;
  bool have_acc = a.accumulation_counter && acc_delta(a.accumulation_counter, b.accumulation_counter,
                                                      false, &dacc) && dacc > 0;
  if (have_acc && a.has_residency && b.has_residency) {
    auto pct = [&](uint64_t x0, uint64_t x1) {
      uint64_t dd = 0;
      return acc_delta(x0, x1, false, &dd) ? std::min(100.0, dd * 100.0 / dacc) : kNaN;
    };
    out->ppt_violation_pct = pct(a.ppt_res, b.ppt_res);
    out->thermal_violation_pct = pct(a.socket_thm_res, b.socket_thm_res);
    out->prochot_violation_pct = pct(a.prochot_res, b.prochot_res);
    out->vr_thm_violation_pct = pct(a.vr_thm_res, b.vr_thm_res);
    out->hbm_thm_violation_pct = pct(a.hbm_thm_res, b.hbm_thm_res);
  }
  if (have_acc && a.has_activity_acc && b.has_activity_acc) {
    uint64_t dg = 0, dm = 0;
    if (acc_delta(a.gfx_activity_acc, b.gfx_activity_acc, true, &dg))
      out->gfx_activity_avg_pct = std::min(100.0, dg * cfg.activity_acc_scale / dacc);
    if (acc_delta(a.mem_activity_acc, b.mem_activity_acc, true, &dm))
      out->mem_activity_avg_pct = std::min(100.0, dm * cfg.activity_acc_scale / dacc);
  }
  if (have_acc && a.has_pcie_bw_acc && b.has_pcie_bw_acc) {
    // pcie_bandwidth_acc adds the instantaneous bandwidth once per accumulation tick (1 kHz on
    // MI355X), so its delta over the counter's is the interval mean in firmware units
    uint64_t dp = 0;
    if (acc_delta(a.pcie_bw_acc, b.pcie_bw_acc, false, &dp))
      out->pcie_Bps = static_cast<double>(dp) * cfg.pcie_bw_unit_bytes / static_cast<double>(dacc);
  }
  if (have_acc) {
    int nx = std::min(a.n_xcd_acc, b.n_xcd_acc);
    out->n_xcd = nx;
    for (int k = 0; k < nx; ++k) {
      uint64_t dx = 0;
      out->xcd_busy_avg[k] = acc_delta(a.xcd_busy_acc[k], b.xcd_busy_acc[k], false, &dx)
                                 ? std::min(100.0, dx * cfg.activity_acc_scale / dacc)
                                 : kNaN;
    }
    if (a.has_xcd_limit_acc && b.has_xcd_limit_acc) {
      out->has_xcd_limit = true;
      auto pct = [&](uint64_t x0, uint64_t x1) {
        uint64_t d = 0;
        return acc_delta(x0, x1, false, &d) ? std::min(100.0, 100.0 * static_cast<double>(d) / dacc) : kNaN;
      };
      for (int k = 0; k < nx; ++k) {
        out->xcd_below_ppt_pct[k] = pct(a.xcd_below_ppt_acc[k], b.xcd_below_ppt_acc[k]);
        out->xcd_below_thm_pct[k] = pct(a.xcd_below_thm_acc[k], b.xcd_below_thm_acc[k]);
        out->xcd_below_total_pct[k] = pct(a.xcd_below_total_acc[k], b.xcd_below_total_acc[k]);
        out->xcd_low_util_pct[k] = pct(a.xcd_low_util_acc[k], b.xcd_low_util_acc[k]);
      }
    }
  }
  int nl = std::min(a.n_links_acc, b.n_links_acc);
  out->n_links = nl;
  for (int k = 0; k < nl; ++k) {
    uint64_t dr = 0, dw = 0;
    out->xgmi_rd_Bps[k] =
        acc_delta(a.xgmi_rd_kb[k], b.xgmi_rd_kb[k], false, &dr) ? dr * cfg.xgmi_kb_bytes / dt : kNaN;
    out->xgmi_wr_Bps[k] =
        acc_delta(a.xgmi_wr_kb[k], b.xgmi_wr_kb[k], false, &dw) ? dw * cfg.xgmi_kb_bytes / dt : kNaN;
  }
}

}  // namespace gpumon
