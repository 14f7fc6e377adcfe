// MI355X-shaped gpu_metrics v1.8 table shared by the fake libamd_smi and fake librocm_smi.
// Both libraries return the same SMU table under the same field names, so one template fills
// amdsmi_gpu_metrics_t and rsmi_gpu_metrics_t. `n` is the per-device call count: accumulators
// advance by one simulated second per call so rates are checkable.
#pragma once

#include <cstdint>
#include <cstring>

namespace fake {

template <typename M>
void fill_metrics(M* m, int d, uint64_t n) {
  memset(m, 0xFF, sizeof *m);  // every field N/A unless set below (firmware convention)
  m->common_header.format_revision = 1;
  m->common_header.content_revision = 8;
  m->temperature_hotspot = static_cast<uint16_t>(46 + d);
  m->temperature_mem = 33;
  m->temperature_vrsoc = 43;
  m->average_gfx_activity = 37;
  m->average_umc_activity = 12;
  m->current_socket_power = 600;
  m->energy_accumulator = 1000000 + n * 1000000;  // x15.3 uJ per tick
  m->system_clock_counter = n * 1000000000ull;     // 1 s per tick (driver ns)
  m->firmware_timestamp = n * 100000000ull;
  m->current_gfxclk = 2100;
  m->current_uclk = 2000;
  m->current_socclk = 1200;
  m->throttle_status = 0;
  m->pcie_link_width = 16;
  m->pcie_link_speed = 320;
  m->pcie_bandwidth_inst = 18;                                   // idle MI355X: 18-21 units
  m->pcie_bandwidth_acc = n * 1000ull * (500000ull + 1000ull * d);  // 1000 ticks per call: 51.2 (+0.1 d) GB/s
  m->pcie_replay_count_acc = 0;
  m->gfx_activity_acc = static_cast<uint32_t>(n * 37 * 1000);  // 37 % per counter tick
  m->mem_activity_acc = static_cast<uint32_t>(n * 12 * 1000);
  m->accumulation_counter = n * 1000;
  m->ppt_residency_acc = n * 100;  // 10 % PVIOL
  m->prochot_residency_acc = 0;
  m->socket_thm_residency_acc = 0;
  m->vr_thm_residency_acc = 0;
  m->hbm_thm_residency_acc = 0;
  m->xgmi_link_speed = 38;
  m->xgmi_link_width = 16;
  m->vram_max_bandwidth = 8192;
  m->num_partition = 1;
  for (int k = 0; k < 8; ++k) {
    m->current_gfxclks[k] = static_cast<uint16_t>(2100 - k);
    m->xcp_stats[0].gfx_busy_inst[k] = 37;
    m->xcp_stats[0].gfx_busy_acc[k] = n * 37 * 1000;
    m->xcp_stats[0].gfx_below_host_limit_ppt_acc[k] = n * 250;    // 25 % of the 1000 ticks per call
    m->xcp_stats[0].gfx_below_host_limit_thm_acc[k] = 0;
    m->xcp_stats[0].gfx_below_host_limit_total_acc[k] = n * 250;
    m->xcp_stats[0].gfx_low_utilization_acc[k] = 0;
  }
  m->xgmi_link_status[0] = 0xFFFF;  // slot 0: N/A on MI355X
  m->xgmi_read_data_acc[0] = 0;
  m->xgmi_write_data_acc[0] = 0;
  for (int k = 1; k < 8; ++k) {
    m->xgmi_link_status[k] = 1;
    m->xgmi_read_data_acc[k] = n * 1000000ull * k;  // k GB/s (KB units, 1 s per tick)
    m->xgmi_write_data_acc[k] = n * 500000ull * k;
  }
}

}  // namespace fake
