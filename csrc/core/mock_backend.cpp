// MockBackend: N scripted fake MI355X devices.
//
// The reference has no fake backend and no tests at all; this backend is what
// lets the whole pipeline (sampler -> attribution -> render -> HTTP) run and be tested on a CPU
// box: BASELINE config #1 "mock backend, 1 fake GPU, Prometheus /metrics on CPU".
// Values follow MI355X shapes: 288 GiB HBM3E, 8 XCDs, 7 xGMI peer links, 1400 W limit.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <thread>

#include "backend.h"
#include "common.h"

namespace gpumon {

static const char* kFieldNames[F_COUNT] = {
    "gfx_util",      "umc_util",       "mm_util",        "vram_used",      "vram_total",
    "gtt_used",      "temp_edge",      "temp_hotspot",   "temp_mem",       "temp_vrgfx",
    "temp_vrsoc",    "temp_vrmem",     "power_cur",      "power_avg",      "power_limit",
    "energy_j",      "gfxclk_cur",     "gfxclk_avg",     "socclk_cur",     "uclk_cur",
    "vclk0_cur",     "dclk0_cur",      "throttle_status", "indep_throttle", "fan_rpm",
    "pcie_width",    "pcie_speed_gts", "pcie_bw_inst",   "pcie_replay",    "pcie_l0_recov",
    "pcie_nak_sent", "pcie_nak_rcvd",  "volt_soc",       "volt_gfx",       "volt_mem",
    "xgmi_link_width", "xgmi_link_speed", "vram_max_bw", "num_partition",  "gfxclk_lock",
    "cu_occupancy"};

int field_by_name(const std::string& name) {
  for (int i = 0; i < F_COUNT; ++i)
    if (name == kFieldNames[i]) return i;
  return -1;
}
const char* field_name(int f) { return (f >= 0 && f < F_COUNT) ? kFieldNames[f] : "?"; }

MockBackend::MockBackend(MockConfig cfg) : cfg_(std::move(cfg)) {}

bool MockBackend::init(std::string* err) {
  std::lock_guard<std::mutex> g(mu_);
  if (cfg_.gpus < 0 || cfg_.gpus > 64) {
    if (err) *err = "mock: gpus must be in [0, 64]";
    return false;
  }
  devs_.clear();
  for (int i = 0; i < cfg_.gpus; ++i) {
    char buf[64];
    snprintf(buf, sizeof buf, "0000:%02x:%02x.0", 0x05 + 0x20 * (i % 8), i / 8);  // 8 buses, then devices
    if (!keep(i, buf)) continue;
    DeviceStatic d;
    d.bdf = buf;
    d.index = static_cast<int>(devs_.size());
    d.hip_id = i;
    d.gpu_id = std::to_string(i);
    snprintf(buf, sizeof buf, "mock-%04x-0000-1000-80d2-%012llx", 0x75a3 + i,
             static_cast<unsigned long long>(cfg_.seed * 1000 + i));
    d.uuid = buf;
    d.model = "AMD Instinct MI355 OAM (mock)";
    d.serial = "MOCK" + std::to_string(i);
    d.gfx_target = "gfx950";
    d.compute_partition = "SPX";
    d.memory_partition = "NPS1";
    d.driver_version = "mock";
    d.driver_source = "library";
    d.vram_total_bytes = 294896.0 * 1048576.0;
    d.power_limit_w = 1400.0;
    d.num_cu = 256;
    d.num_xcc = cfg_.n_xcd;
    d.drm_card = i;
    d.drm_render = 128 + i;
    devs_.push_back(d);
  }
  size_t n = devs_.size();
  forced_util_.assign(n, kNaN);
  forced_xgmi_.assign(n * kMaxLinks, kNaN);
  link_down_.assign(n * kMaxLinks, 0);
  link_calls_.assign(n, 0);
  link_fail_.assign(n, 0);
  frozen_tick_.assign(n, -1);
  scan_fail_.assign(n, 0);
  procs_fail_.assign(n, 0);
  procs_calls_.assign(n, 0);
  calls_.assign(n, 0);
  prewarms_.assign(n, 0);
  energy_.assign(n, 1000000);
  xgmi_rd_.assign(n * kMaxLinks, 0);
  xgmi_wr_.assign(n * kMaxLinks, 0);
  busy_acc_.assign(n * kMaxXcc, 0);
  lim_acc_.assign(n * kMaxXcc * 4, 0);
  acc_counter_.assign(n, 100000);  // 1 s of firmware uptime: a live counter is never 0
  gfx_act_acc_.assign(n, 0);
  pcie_acc_.assign(n, 0);
  t0_ns_ = mono_ns();
  last_ns_.assign(n, t0_ns_);
  // RAS: the blocks MI355X publishes under ras/aca_* (measured), all clean
  ras_.assign(n, RasSample{});
  for (auto& r : ras_) {
    r.valid = true;
    r.source = "mock";
    for (const char* b : {"gfx", "jpeg", "mmhub", "sdma", "umc", "vcn", "xgmi_wafl"}) {
      RasCount c;
      c.block = b;
      c.has_de = true;
      r.blocks.push_back(c);
    }
    r.fatal = r.poison_created = r.poison_consumed = r.bad_pages = 0;
  }
  return true;
}

void MockBackend::sample_ras(int i, DeviceSample* out, int slice, int) {
  if (slice != 0) return;  // whole refresh once per cycle (carried over between)
  std::lock_guard<std::mutex> g(mu_);
  if (i < 0 || i >= static_cast<int>(ras_.size())) return;
  out->ras = ras_[i];
}

void MockBackend::add_ecc(int dev, const std::string& block, uint64_t ue, uint64_t ce, uint64_t de) {
  std::lock_guard<std::mutex> g(mu_);
  if (dev < 0 || dev >= static_cast<int>(ras_.size())) return;
  for (auto& c : ras_[dev].blocks)
    if (c.block == block) {
      c.ue += ue;
      c.ce += ce;
      c.de += de;
      return;
    }
  RasCount c;
  c.block = block;
  c.ue = ue;
  c.ce = ce;
  c.de = de;
  c.has_de = true;
  ras_[dev].blocks.push_back(c);
}

void MockBackend::set_ras_event(int dev, const std::string& event, double value) {
  std::lock_guard<std::mutex> g(mu_);
  if (dev < 0 || dev >= static_cast<int>(ras_.size())) return;
  auto& r = ras_[dev];
  if (event == "fatal") r.fatal = value;
  else if (event == "poison_created") r.poison_created = value;
  else if (event == "poison_consumed") r.poison_consumed = value;
  else if (event == "bad_pages") r.bad_pages = value;
}

void MockBackend::set_util(int dev, double pct) {
  std::lock_guard<std::mutex> g(mu_);
  if (dev >= 0 && dev < static_cast<int>(forced_util_.size())) forced_util_[dev] = pct;
}
void MockBackend::set_procs(const std::vector<MockProc>& procs) {
  std::lock_guard<std::mutex> g(mu_);
  cfg_.procs = procs;
}
void MockBackend::set_fail(int dev, int every) {
  std::lock_guard<std::mutex> g(mu_);
  cfg_.fail_device = dev;
  cfg_.fail_every = every;
}
void MockBackend::set_xgmi(int dev, int link, double gbps) {
  std::lock_guard<std::mutex> g(mu_);
  if (dev < 0 || link < 0 || link >= kMaxLinks) return;
  const size_t k = static_cast<size_t>(dev) * kMaxLinks + link;
  if (k < forced_xgmi_.size()) forced_xgmi_[k] = gbps < 0 ? kNaN : gbps;
}

void MockBackend::set_hang_ms(double ms, int dev) {
  std::lock_guard<std::mutex> g(mu_);
  cfg_.hang_ms = ms;
  cfg_.hang_device = dev;
}
void MockBackend::set_link_up(int dev, int link, bool up) {
  std::lock_guard<std::mutex> g(mu_);
  const size_t k = static_cast<size_t>(dev) * kMaxLinks + link;
  if (dev >= 0 && link >= 0 && link < kMaxLinks && k < link_down_.size()) link_down_[k] = up ? 0 : 1;
}
uint64_t MockBackend::link_calls(int dev) const {
  std::lock_guard<std::mutex> g(mu_);
  return dev >= 0 && dev < static_cast<int>(link_calls_.size()) ? link_calls_[dev] : 0;
}
bool MockBackend::prewarm(int i) {
  std::lock_guard<std::mutex> g(mu_);
  if (i < 0 || i >= static_cast<int>(prewarms_.size())) return false;
  prewarms_[i]++;
  return true;
}
uint64_t MockBackend::prewarms(int dev) const {
  std::lock_guard<std::mutex> g(mu_);
  return dev >= 0 && dev < static_cast<int>(prewarms_.size()) ? prewarms_[dev] : 0;
}
uint64_t MockBackend::calls(int dev) const {
  std::lock_guard<std::mutex> g(mu_);
  return dev >= 0 && dev < static_cast<int>(calls_.size()) ? calls_[dev] : 0;
}

static double mock_util(const MockConfig& c, int dev, double t) {
  if (c.mode == "idle") return 0.0;
  if (c.mode == "load") return 100.0;
  if (c.mode == "const") return c.const_util;
  double u = 50.0 + 45.0 * std::sin(0.7 * t + 1.3 * dev);
  return std::floor(std::max(0.0, std::min(100.0, u)));
}

void MockBackend::sample(int i, DeviceSample* out) {
  out->reset();
  int64_t t0 = mono_ns();
  double hang;
  {
    std::lock_guard<std::mutex> g(mu_);
    hang = (cfg_.hang_device < 0 || cfg_.hang_device == devs_[i].hip_id) ? cfg_.hang_ms : 0.0;
  }
  if (hang > 0) std::this_thread::sleep_for(std::chrono::microseconds(static_cast<int64_t>(hang * 1000)));
  std::lock_guard<std::mutex> g(mu_);
  uint64_t call = ++calls_[i];
  out->host_mono_ns = mono_ns();
  out->host_wall_ns = wall_ns();
  if ((cfg_.fail_device == devs_[i].hip_id || cfg_.fail_device == -2) &&  // -2: every device
      (cfg_.fail_every < 0 || (cfg_.fail_every > 0 && call % static_cast<uint64_t>(cfg_.fail_every) == 0))) {
    out->ok = false;
    out->errors = 1;
    out->last_error = "gpu_metrics: MOCK_INJECTED_FAILURE";
    out->sample_ns = mono_ns() - t0;
    record_call(kCallMetrics, out->sample_ns, false);
    return;
  }
  double t = (out->host_mono_ns - t0_ns_) * 1e-9;
  double util = has(forced_util_[i]) ? forced_util_[i] : mock_util(cfg_, devs_[i].hip_id, t);
  auto& v = out->v;
  v[F_GFX_UTIL] = util;
  v[F_UMC_UTIL] = std::floor(util * 0.6);
  v[F_VRAM_TOTAL] = devs_[i].vram_total_bytes;
  double used = 283.0 * 1048576.0;
  for (const auto& p : cfg_.procs)
    if (p.device == devs_[i].hip_id) used += p.vram_bytes;
  v[F_VRAM_USED] = used;
  v[F_GTT_USED] = 23.0 * 1048576.0;
  v[F_TEMP_HOTSPOT] = 40.0 + util * 0.45;
  v[F_TEMP_MEM] = 33.0 + util * 0.25;
  v[F_TEMP_VRSOC] = 38.0 + util * 0.2;
  double power = 250.0 + util * 11.0;
  v[F_POWER_CUR] = power;
  v[F_POWER_LIMIT] = devs_[i].power_limit_w;
  v[F_GFXCLK_CUR] = util > 0 ? 2100.0 : 95.0;
  v[F_SOCCLK_CUR] = 1200.0;
  v[F_UCLK_CUR] = 2000.0;
  v[F_PCIE_WIDTH] = 16;
  v[F_PCIE_SPEED_GTS] = 32.0;
  // firmware PCIe bandwidth units (x RateConfig::pcie_bw_unit_bytes): idle 18, +100 per % busy
  const double pcie_units = 18.0 + 100.0 * util;
  v[F_PCIE_BW_INST] = pcie_units;
  v[F_PCIE_REPLAY] = 0;
  v[F_PCIE_L0_RECOV] = 0;
  v[F_XGMI_LINK_WIDTH] = 16;
  v[F_XGMI_LINK_SPEED] = 38;
  v[F_VRAM_MAX_BW] = 8192;
  v[F_NUM_PARTITION] = 1;
  v[F_THROTTLE_STATUS] = 0;

  // Accumulators advance with the firmware's table time, in quanta of 1/firmware_hz (as on
  // hardware: a read between two firmware refreshes returns the same accumulators), while the
  // driver stamps system_clock_counter at the read itself.
  Accumulators& a = out->acc;
  a.valid = true;
  int64_t now = out->host_mono_ns;
  uint64_t fw_tick = static_cast<uint64_t>(t * cfg_.firmware_hz);
  if (frozen_tick_[i] >= 0) fw_tick = static_cast<uint64_t>(frozen_tick_[i]);
  const int64_t fw_ns = t0_ns_ + static_cast<int64_t>(fw_tick / std::max(1e-3, cfg_.firmware_hz) * 1e9);
  double elapsed = std::max(0.0, (fw_ns - last_ns_[i]) * 1e-9);
  last_ns_[i] = std::max(last_ns_[i], fw_ns);
  a.firmware_ts = (fw_tick + 1) * static_cast<uint64_t>(1e8 / std::max(1e-3, cfg_.firmware_hz));
  a.system_clock_ns = static_cast<uint64_t>(now);
  energy_[i] += static_cast<uint64_t>(power * elapsed / 15.3e-6);
  a.energy = energy_[i];
  a.energy_resolution_uj = 15.3;
  v[F_ENERGY_J] = static_cast<double>(a.energy) * 15.3e-6;
  acc_counter_[i] += static_cast<uint64_t>(elapsed * 100000.0);  // 10 us units
  a.accumulation_counter = acc_counter_[i];
  a.has_residency = true;
  a.ppt_res = util > 90 ? acc_counter_[i] / 10 : 0;
  a.has_activity_acc = true;
  gfx_act_acc_[i] += static_cast<uint64_t>(util * elapsed * 100000.0);
  a.gfx_activity_acc = gfx_act_acc_[i];
  pcie_acc_[i] += static_cast<uint64_t>(pcie_units * elapsed * 100000.0);
  a.pcie_bw_acc = pcie_acc_[i];
  a.has_pcie_bw_acc = true;
  int nx = cfg_.n_xcd;
  out->n_xcd = nx;
  a.n_xcd_acc = nx;
  for (int k = 0; k < nx && k < kMaxXcc; ++k) {
    double xb = std::max(0.0, std::min(100.0, util + (k - nx / 2) * 0.5));
    out->xcd_busy[k] = std::floor(xb);
    busy_acc_[i * kMaxXcc + k] += static_cast<uint64_t>(xb * elapsed * 100000.0);
    a.xcd_busy_acc[k] = busy_acc_[i * kMaxXcc + k];
    out->gfxclks[k] = v[F_GFXCLK_CUR];
    // residency counters (+1 per 10 us tick while true): PPT-limited above 90 % busy, low
    // utilisation below 5 % (as measured on MI355X: idle = low-util + any)
    const uint64_t ticks = static_cast<uint64_t>(elapsed * 100000.0);
    uint64_t* L = &lim_acc_[(static_cast<size_t>(i) * kMaxXcc + k) * 4];
    const bool ppt = xb > 90.0, low = xb < 5.0;
    if (ppt) L[0] += ticks / 4;
    if (low) L[3] += ticks;
    L[2] += low ? ticks : (ppt ? ticks / 4 : 0);
    a.xcd_below_ppt_acc[k] = L[0];
    a.xcd_below_thm_acc[k] = L[1];
    a.xcd_below_total_acc[k] = L[2];
    a.xcd_low_util_acc[k] = L[3];
  }
  a.has_xcd_limit_acc = nx > 0;
  int nl = std::min(cfg_.n_links + 1, kMaxLinks);  // slot 0 = self, as on MI355X
  out->n_links = nl;
  a.n_links_acc = nl;
  for (int k = 0; k < nl; ++k) {
    if (k > 0) {
      // ~util% of 64 GB/s per link, in KB (or the forced per-link rate)
      const double forced = forced_xgmi_[i * kMaxLinks + k];
      uint64_t kb = static_cast<uint64_t>((has(forced) ? forced : util / 100.0 * 64.0) * 1e6 * elapsed);
      xgmi_rd_[i * kMaxLinks + k] += kb;
      xgmi_wr_[i * kMaxLinks + k] += kb / 2;
    }
    a.xgmi_rd_kb[k] = xgmi_rd_[i * kMaxLinks + k];
    a.xgmi_wr_kb[k] = xgmi_wr_[i * kMaxLinks + k];
    out->links[k].status = k == 0 ? -1 : (link_down_[i * kMaxLinks + k] ? 0 : 1);
    out->links[k].bit_rate_gbps = 38;
  }
  if (cfg_.full)  // fields a real MI355X table leaves N/A get a neutral value
    for (int f = 0; f < F_COUNT; ++f)
      if (!has(v[f])) v[f] = 0.0;
  for (const auto& name : cfg_.unsupported) {
    int f = field_by_name(name);
    if (f >= 0) v[f] = kNaN;
    if (name == "xcd") {
      out->n_xcd = 0;
      a.n_xcd_acc = 0;
    }
    if (name == "xgmi") {
      out->n_links = 0;
      a.n_links_acc = 0;
    }
  }
  out->ok = true;
  out->sample_ns = mono_ns() - t0;
  record_call(kCallMetrics, out->sample_ns, true);
}

bool MockBackend::processes(int i, std::vector<ProcSample>* out) {
  std::lock_guard<std::mutex> g(mu_);
  out->clear();
  if (procs_fail_[i] > 0) {
    --procs_fail_[i];
    return false;
  }
  if (cfg_.procs_fail_every > 0 && ++procs_calls_[i] % static_cast<uint64_t>(cfg_.procs_fail_every) == 0)
    return false;
  double util = has(forced_util_[i]) ? forced_util_[i]
                                     : mock_util(cfg_, devs_[i].hip_id, (mono_ns() - t0_ns_) * 1e-9);
  for (const auto& p : cfg_.procs) {
    if (p.device != devs_[i].hip_id) continue;
    ProcSample ps;
    ps.pid = p.pid;
    ps.name = p.name;
    ps.vram_bytes = p.vram_bytes;
    ps.mem_bytes = p.vram_bytes;
    ps.gtt_bytes = 0;
    ps.cpu_bytes = 0;
    auto key = std::make_pair(p.pid, i);
    // gfx ns advance at util * share of wall time
    uint64_t& ns = proc_gfx_ns_[key];
    ns += static_cast<uint64_t>(util / 100.0 * p.gfx_share * 1e7);
    ps.gfx_ns = ns + static_cast<uint64_t>((mono_ns() - t0_ns_) * (util / 100.0) * p.gfx_share);
    ps.has_gfx_ns = !p.kfd_only;
    if (cfg_.occupancy) ps.cu_occupancy = occ_value(i, p, util);
    ps.queues = p.queues;
    out->push_back(std::move(ps));
  }
  return true;
}

double MockBackend::occ_value(int i, const MockProc& p, double util) {
  if (static_cast<int>(occ_reads_.size()) <= i) occ_reads_.resize(devs_.size(), 0);
  const uint64_t k = occ_reads_[i]++;
  if (i < static_cast<int>(occ_series_.size()) && !occ_series_[i].empty())
    return occ_series_[i][k % occ_series_[i].size()];
  return std::floor(256.0 * util / 100.0 * p.gfx_share);
}

void MockBackend::occupancy(int i, const std::vector<uint32_t>& pids, std::vector<double>* out) {
  std::lock_guard<std::mutex> g(mu_);
  out->assign(pids.size(), kNaN);
  if (i < 0 || i >= static_cast<int>(devs_.size())) return;
  const double util = has(forced_util_[i]) ? forced_util_[i]
                                           : mock_util(cfg_, devs_[i].hip_id, (mono_ns() - t0_ns_) * 1e-9);
  for (size_t k = 0; k < pids.size(); ++k)
    for (const auto& p : cfg_.procs)
      if (p.pid == pids[k] && p.device == devs_[i].hip_id) {
        (*out)[k] = occ_value(i, p, util);
        break;
      }
}

bool MockBackend::occupancy_scan(int i, std::vector<OccRead>* out) {
  std::lock_guard<std::mutex> g(mu_);
  out->clear();
  if (!cfg_.occupancy || i < 0 || i >= static_cast<int>(devs_.size())) return false;
  if (scan_fail_[i] > 0) {
    --scan_fail_[i];
    return false;
  }
  const double util = has(forced_util_[i]) ? forced_util_[i]
                                           : mock_util(cfg_, devs_[i].hip_id, (mono_ns() - t0_ns_) * 1e-9);
  for (const auto& p : cfg_.procs)
    if (p.device == devs_[i].hip_id) {
      OccRead r;
      r.pid = p.pid;
      r.vram_bytes = p.vram_bytes;
      r.cu_occupancy = occ_value(i, p, util);
      out->push_back(r);
    }
  return true;
}

void MockBackend::set_occ_series(int dev, const std::vector<double>& values) {
  std::lock_guard<std::mutex> g(mu_);
  if (dev < 0 || dev >= static_cast<int>(devs_.size())) return;
  if (static_cast<int>(occ_series_.size()) <= dev) occ_series_.resize(devs_.size());
  occ_series_[dev] = values;
  if (static_cast<int>(occ_reads_.size()) <= dev) occ_reads_.resize(devs_.size(), 0);
  occ_reads_[dev] = 0;
}

uint64_t MockBackend::occ_reads(int dev) const {
  std::lock_guard<std::mutex> g(mu_);
  return dev >= 0 && dev < static_cast<int>(occ_reads_.size()) ? occ_reads_[dev] : 0;
}

void MockBackend::sample_links(int i, DeviceSample* out) {
  std::lock_guard<std::mutex> g(mu_);
  if (i >= 0 && i < static_cast<int>(link_calls_.size())) link_calls_[i]++;
  if (i >= 0 && i < static_cast<int>(link_fail_.size()) && link_fail_[i]) {
    out->links_read = -1;  // injected link-metrics failure
    return;
  }
  // one link-metrics entry per table slot (slot 0 = self: no peer), each with the slot's own
  // accumulators; cfg_.link_order scrambles their order like a library that does not list them in
  // table-slot order, cfg_.link_offset gives them another counter origin
  const int nl = std::min(cfg_.n_links + 1, kMaxLinks);
  std::vector<LinkEntry> es;
  for (int k = 0; k < nl; ++k) {
    LinkEntry e;
    if (k == 0) {
      es.push_back(std::move(e));
      continue;
    }
    char buf[32];
    int peer = (devs_[i].hip_id + k) % std::max(2, cfg_.gpus + 1);
    snprintf(buf, sizeof buf, "0000:%02x:00.0", 0x05 + 0x20 * peer);
    const bool down = link_down_[i * kMaxLinks + k] != 0;
    e.peer_bdf = down ? "" : buf;  // a down link reports no peer (as amdsmi does)
    e.bit_rate_gbps = down ? kNaN : 38;
    e.max_bandwidth_gbps = down ? kNaN : 608;
    e.link_type = 2;
    e.has_acc = true;
    const uint64_t off = cfg_.link_offset ? 1000000000ull * static_cast<uint64_t>(k) : 0;
    e.read_kb = xgmi_rd_[i * kMaxLinks + k] + off;
    e.write_kb = xgmi_wr_[i * kMaxLinks + k] + off;
    es.push_back(std::move(e));
  }
  if (cfg_.link_order == "reverse") std::reverse(es.begin(), es.end());
  else if (cfg_.link_order == "rotate" && !es.empty()) std::rotate(es.begin(), es.begin() + 1, es.end());
  out->link_entries = std::move(es);
  out->links_read = 1;
}

void MockBackend::fail_procs(int dev, int n) {
  std::lock_guard<std::mutex> g(mu_);
  if (dev >= 0 && dev < static_cast<int>(procs_fail_.size())) procs_fail_[dev] = n;
}

void MockBackend::fail_scans(int dev, int n) {
  std::lock_guard<std::mutex> g(mu_);
  if (dev >= 0 && dev < static_cast<int>(scan_fail_.size())) scan_fail_[dev] = n;
}

void MockBackend::set_firmware_frozen(int dev, bool frozen) {
  std::lock_guard<std::mutex> g(mu_);
  if (dev < 0 || dev >= static_cast<int>(frozen_tick_.size())) return;
  const double t = (mono_ns() - t0_ns_) * 1e-9;
  frozen_tick_[dev] = frozen ? static_cast<int64_t>(t * cfg_.firmware_hz) : -1;
}

void MockBackend::set_link_fail(int dev, bool fail) {
  std::lock_guard<std::mutex> g(mu_);
  if (dev >= 0 && dev < static_cast<int>(link_fail_.size())) link_fail_[dev] = fail ? 1 : 0;
}

}  // namespace gpumon
