// Firmware gpu_metrics table -> DeviceSample.
//
// libamd_smi (amdsmi_gpu_metrics_t) and rocm_smi_lib (rsmi_gpu_metrics_t) expose the SAME
// SMU/driver table (gpu_metrics v1.x; v1.8 on MI355X) under the same field names, so one template
// converts both. Every firmware field uses the all-ones value of its width as "not available";
// such fields stay NaN and are omitted from the exposition.
#pragma once

#include <cstdint>

#include "sample.h"

namespace gpumon {
namespace mt {

inline double u16v(uint16_t x, double scale = 1.0) { return x == 0xFFFF ? kNaN : static_cast<double>(x) * scale; }
inline double u32v(uint32_t x, double scale = 1.0) {
  return x == 0xFFFFFFFFu ? kNaN : static_cast<double>(x) * scale;
}
inline double u64v(uint64_t x, double scale = 1.0) { return x == ~0ull ? kNaN : static_cast<double>(x) * scale; }
inline bool ok16(uint16_t x) { return x != 0xFFFF; }
inline bool ok32(uint32_t x) { return x != 0xFFFFFFFFu; }
inline bool ok64(uint64_t x) { return x != ~0ull; }

}  // namespace mt

// partition_id selects the XCP block in CPX-style partition modes (falls back to XCP 0).
template <typename M>
void fill_from_gpu_metrics(const M& m, int partition_id, int max_xcp, double power_limit_w,
                           double energy_res_uj, DeviceSample* out) {
  using namespace mt;
  auto& v = out->v;
  v[F_GFX_UTIL] = u16v(m.average_gfx_activity);
  v[F_UMC_UTIL] = u16v(m.average_umc_activity);
  v[F_MM_UTIL] = u16v(m.average_mm_activity);
  v[F_TEMP_EDGE] = u16v(m.temperature_edge);
  v[F_TEMP_HOTSPOT] = u16v(m.temperature_hotspot);
  v[F_TEMP_MEM] = u16v(m.temperature_mem);
  v[F_TEMP_VRGFX] = u16v(m.temperature_vrgfx);
  v[F_TEMP_VRSOC] = u16v(m.temperature_vrsoc);
  v[F_TEMP_VRMEM] = u16v(m.temperature_vrmem);
  for (int k = 0; k < kMaxHbm; ++k) out->hbm_temp[k] = u16v(m.temperature_hbm[k]);
  v[F_POWER_CUR] = u16v(m.current_socket_power);
  v[F_POWER_AVG] = u16v(m.average_socket_power);
  v[F_POWER_LIMIT] = power_limit_w;
  v[F_GFXCLK_CUR] = u16v(m.current_gfxclk);
  v[F_GFXCLK_AVG] = u16v(m.average_gfxclk_frequency);
  v[F_SOCCLK_CUR] = u16v(m.current_socclk);
  v[F_UCLK_CUR] = u16v(m.current_uclk);
  v[F_VCLK0_CUR] = u16v(m.current_vclk0);
  v[F_DCLK0_CUR] = u16v(m.current_dclk0);
  v[F_THROTTLE_STATUS] = u32v(m.throttle_status);
  v[F_INDEP_THROTTLE] = u64v(m.indep_throttle_status);
  v[F_FAN_RPM] = u16v(m.current_fan_speed);
  v[F_PCIE_WIDTH] = u16v(m.pcie_link_width);
  v[F_PCIE_SPEED_GTS] = u16v(m.pcie_link_speed, 0.1);
  v[F_PCIE_BW_INST] = u64v(m.pcie_bandwidth_inst);
  v[F_PCIE_REPLAY] = u64v(m.pcie_replay_count_acc);
  v[F_PCIE_L0_RECOV] = u64v(m.pcie_l0_to_recov_count_acc);
  v[F_PCIE_NAK_SENT] = u32v(m.pcie_nak_sent_count_acc);
  v[F_PCIE_NAK_RCVD] = u32v(m.pcie_nak_rcvd_count_acc);
  v[F_VOLT_SOC] = u16v(m.voltage_soc, 1e-3);
  v[F_VOLT_GFX] = u16v(m.voltage_gfx, 1e-3);
  v[F_VOLT_MEM] = u16v(m.voltage_mem, 1e-3);
  v[F_XGMI_LINK_WIDTH] = u16v(m.xgmi_link_width);
  v[F_XGMI_LINK_SPEED] = u16v(m.xgmi_link_speed);
  v[F_VRAM_MAX_BW] = u64v(m.vram_max_bandwidth);
  v[F_NUM_PARTITION] = u16v(m.num_partition);
  v[F_GFXCLK_LOCK] = u32v(m.gfxclk_lock_status);
  for (int k = 0; k < kMaxGfxClks; ++k) out->gfxclks[k] = u16v(m.current_gfxclks[k]);

  Accumulators& a = out->acc;
  a.valid = true;
  if (ok64(m.energy_accumulator)) {
    a.energy = m.energy_accumulator;
    a.energy_resolution_uj = energy_res_uj;
    v[F_ENERGY_J] = static_cast<double>(a.energy) * energy_res_uj * 1e-6;
  }
  a.firmware_ts = ok64(m.firmware_timestamp) ? m.firmware_timestamp : 0;
  a.system_clock_ns = ok64(m.system_clock_counter) ? m.system_clock_counter : 0;
  if (ok64(m.accumulation_counter)) {
    a.accumulation_counter = m.accumulation_counter;
    a.has_residency = ok64(m.ppt_residency_acc);
    a.prochot_res = ok64(m.prochot_residency_acc) ? m.prochot_residency_acc : 0;
    a.ppt_res = ok64(m.ppt_residency_acc) ? m.ppt_residency_acc : 0;
    a.socket_thm_res = ok64(m.socket_thm_residency_acc) ? m.socket_thm_residency_acc : 0;
    a.vr_thm_res = ok64(m.vr_thm_residency_acc) ? m.vr_thm_residency_acc : 0;
    a.hbm_thm_res = ok64(m.hbm_thm_residency_acc) ? m.hbm_thm_residency_acc : 0;
  }
  if (ok32(m.gfx_activity_acc)) {
    a.has_activity_acc = true;
    a.gfx_activity_acc = m.gfx_activity_acc;
    a.mem_activity_acc = ok32(m.mem_activity_acc) ? m.mem_activity_acc : 0;
  }
  if (ok64(m.pcie_bandwidth_acc)) {
    a.has_pcie_bw_acc = true;
    a.pcie_bw_acc = m.pcie_bandwidth_acc;
  }
  // Per-XCD (XCC) busy: the XCP this device is (partition_id in CPX modes), else XCP 0.
  int xcp = partition_id;
  if (xcp < 0 || xcp >= max_xcp || !ok32(m.xcp_stats[xcp].gfx_busy_inst[0])) xcp = 0;
  const auto& xs = m.xcp_stats[xcp];
  int nx = 0;
  for (int k = 0; k < kMaxXcc; ++k) {
    if (!ok32(xs.gfx_busy_inst[k])) break;
    out->xcd_busy[k] = static_cast<double>(xs.gfx_busy_inst[k]);
    a.xcd_busy_acc[k] = ok64(xs.gfx_busy_acc[k]) ? xs.gfx_busy_acc[k] : 0;
    nx = k + 1;
  }
  if (nx > 0 && ok64(xs.gfx_below_host_limit_total_acc[0])) {
    a.has_xcd_limit_acc = true;
    for (int k = 0; k < nx; ++k) {
      a.xcd_below_ppt_acc[k] = ok64(xs.gfx_below_host_limit_ppt_acc[k]) ? xs.gfx_below_host_limit_ppt_acc[k] : 0;
      a.xcd_below_thm_acc[k] = ok64(xs.gfx_below_host_limit_thm_acc[k]) ? xs.gfx_below_host_limit_thm_acc[k] : 0;
      a.xcd_below_total_acc[k] =
          ok64(xs.gfx_below_host_limit_total_acc[k]) ? xs.gfx_below_host_limit_total_acc[k] : 0;
      a.xcd_low_util_acc[k] = ok64(xs.gfx_low_utilization_acc[k]) ? xs.gfx_low_utilization_acc[k] : 0;
    }
  }
  out->n_xcd = nx;
  a.n_xcd_acc = nx;
  // xGMI accumulators (KB) and link status. Slot 0 on MI355X is the (N/A) self slot.
  int nl = 0;
  for (int k = 0; k < kMaxLinks; ++k) {
    a.xgmi_rd_kb[k] = ok64(m.xgmi_read_data_acc[k]) ? m.xgmi_read_data_acc[k] : 0;
    a.xgmi_wr_kb[k] = ok64(m.xgmi_write_data_acc[k]) ? m.xgmi_write_data_acc[k] : 0;
    out->links[k].status = ok16(m.xgmi_link_status[k]) ? m.xgmi_link_status[k] : -1;
    if (ok16(m.xgmi_link_status[k]) || (ok64(m.xgmi_read_data_acc[k]) && m.xgmi_read_data_acc[k]) ||
        (ok64(m.xgmi_write_data_acc[k]) && m.xgmi_write_data_acc[k]))
      nl = k + 1;
  }
  out->n_links = nl;
  a.n_links_acc = nl;
  if (ok16(m.xgmi_link_speed))
    for (int k = 0; k < nl; ++k) out->links[k].bit_rate_gbps = m.xgmi_link_speed;
}

}  // namespace gpumon
