// Sample records produced by a Backend each tick.
//
// Reference parity: /root/reference/gpu.py:104-109 queries per GPU
//   gpu_uuid, utilization.gpu, utilization.memory, memory.total, memory.used, memory.free
// and gpu.py:111-116 per process pid, process_name, gpu_uuid, used_memory.
// DeviceSample carries those (gfx_util, umc_util, vram_*) plus the MI355X fields the north star
// adds (temperatures, power/energy, clocks, per-XCD busy, xGMI per-link accumulators, PCIe,
// throttle residencies). A field that the device does not support is NaN and is not exported.
#pragma once

#include <array>
#include <cmath>
#include <cstdint>
#include <limits>
#include <string>
#include <vector>

namespace gpumon {

constexpr int kMaxXcc = 8;        // gfx950: 8 XCDs per device in SPX mode
constexpr int kMaxLinks = 8;      // amdsmi AMDSMI_MAX_NUM_XGMI_LINKS (MI355X uses 7 peer links)
constexpr int kMaxHbm = 4;        // AMDSMI_NUM_HBM_INSTANCES
constexpr int kMaxGfxClks = 8;    // AMDSMI_MAX_NUM_GFX_CLKS

constexpr double kNaN = std::numeric_limits<double>::quiet_NaN();
inline bool has(double v) { return !std::isnan(v); }

// Static (per-process-lifetime) identity of a device. Reference used nvidia-smi output order
// as the short id (gpu.py:119-120, quirk Q10); we use amdsmi enumeration hip_id.
struct DeviceStatic {
  int index = 0;             // position in this exporter's device list
  int hip_id = -1;           // matches HIP_VISIBLE_DEVICES order
  int drm_card = -1;
  int drm_render = -1;
  int kfd_node = -1;
  int partition_id = 0;
  std::string gpu_id;        // exported short id label (hip_id as decimal)
  std::string uuid;
  std::string bdf;           // "0000:26:00.0"
  std::string model;         // market name
  std::string serial;
  std::string gfx_target;    // "gfx950"
  std::string compute_partition;  // SPX / CPX ...
  std::string memory_partition;   // NPS1 ...
  std::string driver_version;
  std::string driver_source;  // module | kernel | library (common.h driver_version_label)
  double vram_total_bytes = kNaN;
  double power_limit_w = kNaN;
  int num_cu = 0;
  int num_xcc = 0;
};

// Scalar fields of one device sample. NaN = not supported / not read.
enum Field : int {
  F_GFX_UTIL = 0,       // % (gfx_activity)               -> node_gpu.gpu_util (gpu.py:138)
  F_UMC_UTIL,           // % memory controller activity   -> reference queried utilization.memory (gpu.py:105) but never emitted
  F_MM_UTIL,            // % multimedia
  F_VRAM_USED,          // bytes                          -> node_gpu.mem_used (gpu.py:139)
  F_VRAM_TOTAL,         // bytes                          -> node_gpu.mem_total (gpu.py:140)
  F_GTT_USED,           // bytes
  F_TEMP_EDGE,          // C
  F_TEMP_HOTSPOT,
  F_TEMP_MEM,
  F_TEMP_VRGFX,
  F_TEMP_VRSOC,
  F_TEMP_VRMEM,
  F_POWER_CUR,          // W
  F_POWER_AVG,          // W (firmware average)
  F_POWER_LIMIT,        // W
  F_ENERGY_J,           // J (accumulator * resolution)
  F_GFXCLK_CUR,         // MHz
  F_GFXCLK_AVG,
  F_SOCCLK_CUR,
  F_UCLK_CUR,
  F_VCLK0_CUR,
  F_DCLK0_CUR,
  F_THROTTLE_STATUS,    // bitfield
  F_INDEP_THROTTLE,     // bitfield
  F_FAN_RPM,
  F_PCIE_WIDTH,         // lanes
  F_PCIE_SPEED_GTS,     // GT/s
  F_PCIE_BW_INST,       // bytes/s instantaneous (firmware units x RateConfig::pcie_bw_unit_bytes, set in tick())
  F_PCIE_REPLAY,        // count
  F_PCIE_L0_RECOV,      // count
  F_PCIE_NAK_SENT,
  F_PCIE_NAK_RCVD,
  F_VOLT_SOC,           // V
  F_VOLT_GFX,
  F_VOLT_MEM,
  F_XGMI_LINK_WIDTH,
  F_XGMI_LINK_SPEED,    // Gb/s per lane (bit rate)
  F_VRAM_MAX_BW,        // GB/s
  F_NUM_PARTITION,
  F_GFXCLK_LOCK,
  F_CU_OCC,             // CUs holding waves, summed over the device's processes (KFD cu_occupancy)
  F_COUNT
};

// Raw accumulators used for rate computation (kept exact as integers).
struct Accumulators {
  bool valid = false;
  uint64_t energy = 0;               // energy_accumulator raw counts
  double energy_resolution_uj = 15.259;  // uJ per count
  uint64_t accumulation_counter = 0;     // throttle residency time base
  uint64_t prochot_res = 0, ppt_res = 0, socket_thm_res = 0, vr_thm_res = 0, hbm_thm_res = 0;
  bool has_residency = false;
  uint64_t gfx_activity_acc = 0;     // uint32 in firmware, widened
  uint64_t mem_activity_acc = 0;
  bool has_activity_acc = false;
  uint64_t pcie_bw_acc = 0;
  bool has_pcie_bw_acc = false;
  std::array<uint64_t, kMaxXcc> xcd_busy_acc{};
  int n_xcd_acc = 0;
  // gpu_metrics v1.8 xcp_stats v1.2 per-XCC residency counters: +1 per accumulation tick while
  // the XCC clock is held below the host limit by PPT / thermal / any reason, or the XCC is in
  // low utilisation (measured on MI355X: idle 1.0/tick low-util + any; bf16 burn 0).
  std::array<uint64_t, kMaxXcc> xcd_below_ppt_acc{}, xcd_below_thm_acc{}, xcd_below_total_acc{}, xcd_low_util_acc{};
  bool has_xcd_limit_acc = false;
  std::array<uint64_t, kMaxLinks> xgmi_rd_kb{};
  std::array<uint64_t, kMaxLinks> xgmi_wr_kb{};
  int n_links_acc = 0;
  uint64_t firmware_ts = 0;          // 10 ns units
  uint64_t system_clock_ns = 0;      // driver-attached ns
};

struct LinkInfo {
  std::string peer_bdf;
  double bit_rate_gbps = kNaN;       // per-lane Gb/s
  double max_bandwidth_gbps = kNaN;  // link max, Gb/s
  int link_type = -1;
  int status = -1;                   // 0 down, 1 up, 2 disabled
};

// One entry of amdsmi_get_link_metrics (amdsmi.h amdsmi_link_metrics_t.links[]): peer identity
// and per-link read / write KB in the same struct. Its ORDER is not the gpu_metrics table's xGMI
// slot order (7 entries vs 8 slots on MI355X), so the exporter pairs entries with slots by their
// accumulators (xgmi_map.h) before the identity lands on a slot's LinkInfo.
struct LinkEntry {
  std::string peer_bdf;              // "" = self / unknown
  uint64_t read_kb = 0, write_kb = 0;
  bool has_acc = false;
  double bit_rate_gbps = kNaN;
  double max_bandwidth_gbps = kNaN;
  int link_type = -1;
};

// RAS / ECC error counters of one device (refreshed every `ras_every` ticks; the reference has no
// health data at all). Source: the kernel's ras/ sysfs files (aca_<block> on MI300/MI355X, or
// <block>_err_count), else amdsmi_get_gpu_ecc_count per block.
struct RasCount {
  std::string block;       // umc, gfx, sdma, mmhub, xgmi_wafl, vcn, jpeg, ...
  uint64_t ue = 0, ce = 0, de = 0;  // uncorrectable, correctable, deferred (accumulated)
  bool has_de = false;
};

struct RasSample {
  bool valid = false;
  std::string source;      // "sysfs" | "amdsmi" | "mock"
  std::vector<RasCount> blocks;
  double fatal = kNaN, poison_created = kNaN, poison_consumed = kNaN;  // ras/event_state counts
  double bad_pages = kNaN; // retired / pending VRAM pages (ras/gpu_vram_bad_pages entries)
  int stale_items = 0;     // files due in this read that failed (their last values are carried)
};

struct DeviceSample {
  bool ok = false;                  // at least the primary metrics call succeeded
  bool fresh = true;                // firmware table advanced since last tick
  int64_t host_mono_ns = 0;
  int64_t host_wall_ns = 0;
  int64_t sample_ns = 0;            // time spent sampling this device
  std::array<double, F_COUNT> v;
  std::array<double, kMaxXcc> xcd_busy;      // % instantaneous per XCD
  std::array<double, kMaxGfxClks> gfxclks;   // MHz per XCD clock domain
  std::array<double, kMaxHbm> hbm_temp;
  int n_xcd = 0;
  int n_links = 0;
  std::array<LinkInfo, kMaxLinks> links;
  std::vector<LinkEntry> link_entries;  // raw link-metrics entries, on a link-refresh tick only
  int links_read = 0;                   // this tick's link-metrics read: 1 ok, -1 failed, 0 not made
  int procs_read = 0;                   // this tick's process list: 1 ok, -1 failed, 0 not made/unsupported
  bool procs_held = false;              // the process list is the last good one (procs_read -1)
  Accumulators acc;
  RasSample ras;                    // valid only on ticks that refreshed it (carried over otherwise)
  uint32_t errors = 0;              // failed calls this tick
  std::string last_error;

  DeviceSample() { reset(); }
  void reset() {
    ok = false;
    fresh = true;
    v.fill(kNaN);
    xcd_busy.fill(kNaN);
    gfxclks.fill(kNaN);
    hbm_temp.fill(kNaN);
    n_xcd = 0;
    n_links = 0;
    for (auto& l : links) l = LinkInfo{};
    link_entries.clear();
    links_read = 0;
    procs_read = 0;
    procs_held = false;
    acc = Accumulators{};
    ras = RasSample{};
    errors = 0;
    last_error.clear();
  }
};

// One GPU process on one device (reference: gpu.py:111-116, amdsmi_proc_info_t here).
struct ProcSample {
  uint32_t pid = 0;
  std::string name;
  double vram_bytes = kNaN;
  double gtt_bytes = kNaN;
  double cpu_bytes = kNaN;
  double mem_bytes = kNaN;
  uint64_t gfx_ns = 0;          // accumulated gfx engine time
  bool has_gfx_ns = false;
  // KFD stats_<gpu>/cu_occupancy: the process's resident waves / max waves per CU ("CU-equivalents
  // of waves"; 256 = every wave slot of an MI355X held). Instantaneous when read once; the device
  // worker also reads it `occ_samples - 1` more times between ticks and stores the interval mean.
  double cu_occupancy = kNaN;
  int occ_samples = 0;          // reads behind cu_occupancy (0 = none)
  int occ_busy = 0;             // of those, reads with waves resident (> 0): the process's busy share
  // Hardware (user-mode) queues the process holds on this device, from KFD's per-process queue list
  // (sysfs fast path); -1 = unknown. 0 = a context that never submitted work here: the peer context
  // of a multi-GPU process (pod_rows.cpp).
  int queues = -1;
};

// One between-ticks KFD read of a process on a device (Backend::occupancy_scan): lists processes
// that arrived since the last tick too, so a new tenant is sub-sampled from its first interval.
struct OccRead {
  uint32_t pid = 0;
  double cu_occupancy = kNaN;
  double vram_bytes = kNaN;
};

// Derived per-device values computed from two consecutive samples.
struct DeviceRates {
  bool valid = false;
  double dt_s = 0;
  double power_from_energy_w = kNaN;
  double ppt_violation_pct = kNaN;
  double thermal_violation_pct = kNaN;
  double prochot_violation_pct = kNaN;
  double vr_thm_violation_pct = kNaN;
  double hbm_thm_violation_pct = kNaN;
  double gfx_activity_avg_pct = kNaN;
  double mem_activity_avg_pct = kNaN;
  std::array<double, kMaxXcc> xcd_busy_avg{};
  int n_xcd = 0;
  // % of the interval each XCC clock spent below the host limit (by reason) / in low utilisation
  std::array<double, kMaxXcc> xcd_below_ppt_pct{}, xcd_below_thm_pct{}, xcd_below_total_pct{}, xcd_low_util_pct{};
  bool has_xcd_limit = false;
  std::array<double, kMaxLinks> xgmi_rd_Bps{};
  std::array<double, kMaxLinks> xgmi_wr_Bps{};
  int n_links = 0;
  // PCIe bandwidth over the interval, both directions (bytes/s): d(pcie_bandwidth_acc) over the
  // firmware's accumulation ticks (rates.cpp; unit measured on MI355X, docs/metrics.md)
  double pcie_Bps = kNaN;
};

}  // namespace gpumon
