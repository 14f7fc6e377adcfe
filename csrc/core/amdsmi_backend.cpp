// AmdSmiBackend: direct libamd_smi sampling for MI355X (gfx950).
//
// Reference parity: replaces `nvidia-smi --query-gpu=...` and `--query-compute-apps=...`
// subprocesses (/root/reference/gpu.py:104-116) with in-process calls. One tick per device costs
// one amdsmi_get_gpu_metrics_info (the firmware table: activity, clocks, temps, power, energy,
// per-XCD busy, xGMI accumulators, PCIe, throttle residencies; ~0.3 ms measured on MI355X) +
// amdsmi_get_gpu_vram_usage (~0.1 ms) + amdsmi_get_gpu_process_list (~0.7 ms). The slow
// amdsmi_get_violation_status (~100 ms measured) is deliberately NOT used: the same residency
// accumulators are in the metrics table and rates are derived from them (rates.cpp).
#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "backend.h"
#include "common.h"
#include "metrics_table.h"
#include "ras.h"
#include "smi_table.h"
#include "sysfs_fast.h"

namespace gpumon {

// ---------------------------------------------------------------------------------------------
// SmiTable
// ---------------------------------------------------------------------------------------------
bool SmiTable::load(const std::string& explicit_path, std::string* err) {
  if (dl) return true;
  std::vector<std::string> candidates;
  if (!explicit_path.empty()) candidates.push_back(explicit_path);
  if (const char* e = getenv("GPUMON_AMDSMI_LIB")) candidates.emplace_back(e);
  candidates.emplace_back("libamd_smi.so.26");
  candidates.emplace_back("libamd_smi.so");
  if (const char* r = getenv("ROCM_PATH")) candidates.push_back(std::string(r) + "/lib/libamd_smi.so");
  candidates.emplace_back("/opt/rocm/lib/libamd_smi.so.26");
  candidates.emplace_back("/opt/rocm/lib/libamd_smi.so");
  std::string errs;
  for (const auto& c : candidates) {
    dl = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (dl) {
      path = c;
      break;
    }
    const char* e = dlerror();
    errs += c + ": " + (e ? e : "?") + "; ";
  }
  if (!dl) {
    if (err) *err = "cannot dlopen libamd_smi (" + errs + ")";
    return false;
  }
#define GPUMON_REQ(fn)                                                        \
  fn = reinterpret_cast<decltype(fn)>(dlsym(dl, #fn));                        \
  if (!fn) {                                                                  \
    if (err) *err = std::string("libamd_smi missing required symbol ") + #fn; \
    unload();                                                                 \
    return false;                                                             \
  }
  GPUMON_SMI_REQUIRED(GPUMON_REQ)
#undef GPUMON_REQ
#define GPUMON_OPT(fn) fn = reinterpret_cast<decltype(fn)>(dlsym(dl, #fn));
  GPUMON_SMI_OPTIONAL(GPUMON_OPT)
#undef GPUMON_OPT
  return true;
}

void SmiTable::unload() {
  if (dl) dlclose(dl);
  dl = nullptr;
#define GPUMON_NULL(fn) fn = nullptr;
  GPUMON_SMI_REQUIRED(GPUMON_NULL)
  GPUMON_SMI_OPTIONAL(GPUMON_NULL)
#undef GPUMON_NULL
}

const char* smi_status_str(int s) {
  switch (s) {
    case AMDSMI_STATUS_SUCCESS: return "SUCCESS";
    case AMDSMI_STATUS_INVAL: return "INVAL";
    case AMDSMI_STATUS_NOT_SUPPORTED: return "NOT_SUPPORTED";
    case AMDSMI_STATUS_NOT_YET_IMPLEMENTED: return "NOT_YET_IMPLEMENTED";
    case AMDSMI_STATUS_FAIL_LOAD_MODULE: return "FAIL_LOAD_MODULE";
    case AMDSMI_STATUS_NO_PERM: return "NO_PERM";
    case AMDSMI_STATUS_OUT_OF_RESOURCES: return "OUT_OF_RESOURCES";
    case AMDSMI_STATUS_INIT_ERROR: return "INIT_ERROR";
    case AMDSMI_STATUS_NOT_FOUND: return "NOT_FOUND";
    case AMDSMI_STATUS_BUSY: return "BUSY";
    case AMDSMI_STATUS_TIMEOUT: return "TIMEOUT";
    case AMDSMI_STATUS_DRIVER_NOT_LOADED: return "DRIVER_NOT_LOADED";
    default: return "ERROR";
  }
}

// ---------------------------------------------------------------------------------------------
// helpers: firmware N/A sentinels are all-ones of the field width
// ---------------------------------------------------------------------------------------------
static inline double u16v(uint16_t x, double scale = 1.0) {
  return x == 0xFFFF ? kNaN : static_cast<double>(x) * scale;
}
static inline double u32v(uint32_t x, double scale = 1.0) {
  return x == 0xFFFFFFFFu ? kNaN : static_cast<double>(x) * scale;
}
static inline double u64v(uint64_t x, double scale = 1.0) {
  return x == ~0ull ? kNaN : static_cast<double>(x) * scale;
}
// Times one amdsmi call into the backend's per-call accounting (member-function scope only).
#define SMI_TIMED(call_id, expr)                                                                  \
  ([&]() {                                                                                        \
    const int64_t t_start_ = mono_ns();                                                           \
    const amdsmi_status_t s_ = (expr);                                                            \
    record_call(call_id, mono_ns() - t_start_,                                                    \
                s_ == AMDSMI_STATUS_SUCCESS || s_ == AMDSMI_STATUS_OUT_OF_RESOURCES ||             \
                    s_ == AMDSMI_STATUS_NOT_SUPPORTED);                                           \
    return s_;                                                                                    \
  }())

static inline bool ok16(uint16_t x) { return x != 0xFFFF; }
static inline bool ok32(uint32_t x) { return x != 0xFFFFFFFFu; }
static inline bool ok64(uint64_t x) { return x != ~0ull; }

static std::string bdf_str(const amdsmi_bdf_t& b) {
  char buf[32];
  snprintf(buf, sizeof buf, "%04llx:%02llx:%02llx.%llx",
           static_cast<unsigned long long>(b.domain_number),
           static_cast<unsigned long long>(b.bus_number),
           static_cast<unsigned long long>(b.device_number),
           static_cast<unsigned long long>(b.function_number));
  return buf;
}

// ---------------------------------------------------------------------------------------------
// AmdSmiBackend
// ---------------------------------------------------------------------------------------------
AmdSmiBackend::AmdSmiBackend(std::string lib_path) : lib_path_(std::move(lib_path)) {}

AmdSmiBackend::~AmdSmiBackend() { shutdown(); }

void AmdSmiBackend::shutdown() {
  if (t_ && inited_) t_->amdsmi_shut_down();
  inited_ = false;
  handles_.clear();
  devs_.clear();
  caps_.clear();
  fast_.clear();
  kfd_ids_.clear();
}

bool AmdSmiBackend::init(std::string* err) {
  shutdown();
  if (!t_) t_ = std::make_unique<SmiTable>();
  if (!t_->load(lib_path_, err)) return false;
  amdsmi_status_t st = t_->amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    if (err) *err = std::string("amdsmi_init: ") + smi_status_str(st);
    return false;
  }
  inited_ = true;
  if (t_->amdsmi_get_lib_version) {
    amdsmi_version_t v{};
    if (t_->amdsmi_get_lib_version(&v) == AMDSMI_STATUS_SUCCESS)
      lib_version_ = std::to_string(v.major) + "." + std::to_string(v.minor) + "." +
                     std::to_string(v.release);
  }
  uint32_t nsock = 0;
  st = t_->amdsmi_get_socket_handles(&nsock, nullptr);
  if (st != AMDSMI_STATUS_SUCCESS) {
    if (err) *err = std::string("amdsmi_get_socket_handles: ") + smi_status_str(st);
    return false;
  }
  std::vector<amdsmi_socket_handle> socks(nsock);
  if (nsock) t_->amdsmi_get_socket_handles(&nsock, socks.data());
  std::vector<std::pair<int, void*>> found;  // (hip_id, handle)
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t np = 0;
    if (t_->amdsmi_get_processor_handles(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> ph(np);
    if (np && t_->amdsmi_get_processor_handles(socks[s], &np, ph.data()) != AMDSMI_STATUS_SUCCESS)
      continue;
    for (auto h : ph) {
      if (t_->amdsmi_get_processor_type) {
        processor_type_t pt{};
        if (t_->amdsmi_get_processor_type(h, &pt) == AMDSMI_STATUS_SUCCESS &&
            pt != AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          continue;
      }
      int hip = static_cast<int>(found.size());
      if (t_->amdsmi_get_gpu_enumeration_info) {
        amdsmi_enumeration_info_t ei{};
        if (t_->amdsmi_get_gpu_enumeration_info(h, &ei) == AMDSMI_STATUS_SUCCESS && ok32(ei.hip_id))
          hip = static_cast<int>(ei.hip_id);
      }
      found.emplace_back(hip, h);
    }
  }
  std::sort(found.begin(), found.end(),
            [](const auto& a, const auto& b) { return a.first < b.first; });
  for (auto& [hip, h] : found) {
    std::string bdf;
    if (t_->amdsmi_get_gpu_device_bdf) {
      amdsmi_bdf_t b{};
      if (t_->amdsmi_get_gpu_device_bdf(h, &b) == AMDSMI_STATUS_SUCCESS) bdf = bdf_str(b);
    }
    if (!keep(hip, bdf)) continue;
    DeviceStatic d;
    d.bdf = bdf;
    d.index = static_cast<int>(devs_.size());
    d.hip_id = hip;
    d.gpu_id = std::to_string(hip);
    if (t_->amdsmi_get_gpu_enumeration_info) {
      amdsmi_enumeration_info_t ei{};
      if (t_->amdsmi_get_gpu_enumeration_info(h, &ei) == AMDSMI_STATUS_SUCCESS) {
        d.drm_card = ok32(ei.drm_card) ? static_cast<int>(ei.drm_card) : -1;
        d.drm_render = ok32(ei.drm_render) ? static_cast<int>(ei.drm_render) : -1;
      }
    }
    if (t_->amdsmi_get_gpu_device_uuid) {
      char uuid[AMDSMI_MAX_STRING_LENGTH] = {0};
      unsigned int len = sizeof uuid;
      if (t_->amdsmi_get_gpu_device_uuid(h, &len, uuid) == AMDSMI_STATUS_SUCCESS) d.uuid = uuid;
    }
    if (t_->amdsmi_get_gpu_asic_info) {
      amdsmi_asic_info_t ai{};
      if (t_->amdsmi_get_gpu_asic_info(h, &ai) == AMDSMI_STATUS_SUCCESS) {
        d.model = ai.market_name;
        d.serial = ai.asic_serial;
        if (ok32(ai.num_of_compute_units)) d.num_cu = static_cast<int>(ai.num_of_compute_units);
        if (ok64(ai.target_graphics_version)) {
          char gfx[32];
          snprintf(gfx, sizeof gfx, "gfx%llx", static_cast<unsigned long long>(ai.target_graphics_version));
          d.gfx_target = gfx;
        }
      }
    }
    uint64_t kfd_id = 0;
    if (t_->amdsmi_get_gpu_kfd_info) {
      amdsmi_kfd_info_t ki{};
      if (t_->amdsmi_get_gpu_kfd_info(h, &ki) == AMDSMI_STATUS_SUCCESS) {
        kfd_id = ok64(ki.kfd_id) ? ki.kfd_id : 0;
        d.kfd_node = ok32(ki.node_id) ? static_cast<int>(ki.node_id) : -1;
        d.partition_id = ok32(ki.current_partition_id) ? static_cast<int>(ki.current_partition_id) : 0;
      }
    }
    if (t_->amdsmi_get_gpu_compute_partition) {
      char buf[64] = {0};
      if (t_->amdsmi_get_gpu_compute_partition(h, buf, sizeof buf) == AMDSMI_STATUS_SUCCESS)
        d.compute_partition = buf;
    }
    if (t_->amdsmi_get_gpu_memory_partition) {
      char buf[64] = {0};
      if (t_->amdsmi_get_gpu_memory_partition(h, buf, sizeof buf) == AMDSMI_STATUS_SUCCESS)
        d.memory_partition = buf;
    }
    {
      std::string raw, module_version;
      amdsmi_driver_info_t di{};
      if (t_->amdsmi_get_gpu_driver_info && t_->amdsmi_get_gpu_driver_info(h, &di) == AMDSMI_STATUS_SUCCESS)
        raw.assign(di.driver_version, strnlen(di.driver_version, sizeof di.driver_version));
      read_file(sys_root_ + "/module/amdgpu/version", &module_version, 256);
      d.driver_version = driver_version_label(raw, module_version, &d.driver_source);
    }
    if (t_->amdsmi_get_power_info) {
      amdsmi_power_info_t pi{};
      if (t_->amdsmi_get_power_info(h, &pi) == AMDSMI_STATUS_SUCCESS && ok32(pi.power_limit)) {
        // ROCm 7.2 reports power_limit in microwatts despite the header comment (1400000000).
        double pl = static_cast<double>(pi.power_limit);
        d.power_limit_w = pl > 1e5 ? pl / 1e6 : pl;
      }
    }
    if (t_->amdsmi_get_gpu_vram_usage) {
      amdsmi_vram_usage_t vu{};
      if (t_->amdsmi_get_gpu_vram_usage(h, &vu) == AMDSMI_STATUS_SUCCESS)
        d.vram_total_bytes = static_cast<double>(vu.vram_total) * 1048576.0;
    }
    handles_.push_back(h);
    kfd_ids_.push_back(kfd_id);
    devs_.push_back(std::move(d));
    caps_.emplace_back();
    proc_buf_.emplace_back(sizeof(amdsmi_proc_info_t) * 64);
  }
  if (replicate_ > 1 && !devs_.empty()) {
    const size_t real = devs_.size();
    for (int r = 1; r < replicate_; ++r)
      for (size_t k = 0; k < real; ++k) {
        DeviceStatic d = devs_[k];
        d.index = static_cast<int>(devs_.size());
        d.gpu_id = std::to_string(d.index);
        d.model += " (replica of hip " + std::to_string(devs_[k].hip_id) + ")";
        handles_.push_back(handles_[k]);
        kfd_ids_.push_back(kfd_ids_[k]);
        devs_.push_back(std::move(d));
        caps_.emplace_back();
        proc_buf_.emplace_back(sizeof(amdsmi_proc_info_t) * 64);
      }
  }
  if (devs_.empty()) {
    if (err) *err = "amdsmi: no AMD GPUs found (after device filter)";
    return false;
  }
  // Energy resolution is device-global on MI3xx/MI355X; read it once.
  if (t_->amdsmi_get_energy_count) {
    uint64_t e = 0, ts = 0;
    float res = 0;
    if (t_->amdsmi_get_energy_count(handles_[0], &e, &res, &ts) == AMDSMI_STATUS_SUCCESS && res > 0)
      energy_res_uj_ = res;
  }
  // Sysfs fast path: per device, only after its decoded table matches libamd_smi's.
  fast_.clear();
  fast_.resize(devs_.size());
  fast_status_ = fast_path_ ? "" : "disabled by config";
  if (fast_path_) {
    int ok = 0;
    for (size_t i = 0; i < devs_.size(); ++i) {
      auto g = std::make_unique<SysfsGpu>();
      std::string why;
      if (devs_[i].bdf.empty() ||
          !g->open(sys_root_, proc_root_, devs_[i].bdf, kfd_ids_[i], devs_[i].drm_render, &why)) {
        fast_status_ = "gpu " + devs_[i].gpu_id + ": " + (why.empty() ? "no BDF" : why);
        continue;
      }
      fast_[i] = std::move(g);
      if (!validate_fast(static_cast<int>(i), &why)) {
        fast_[i].reset();
        fast_status_ = "gpu " + devs_[i].gpu_id + ": " + why;
        continue;
      }
      ok++;
    }
    if (ok == static_cast<int>(devs_.size())) fast_status_ = "sysfs";
    GPUMON_LOG(ok ? LogLevel::kInfo : LogLevel::kWarn, "amdsmi",
               "sysfs fast path on " + std::to_string(ok) + "/" + std::to_string(devs_.size()) +
                   " GPU(s)" + (ok == static_cast<int>(devs_.size()) ? "" : " (" + fast_status_ + ")"));
  }
  GPUMON_LOG(LogLevel::kInfo, "amdsmi",
             "loaded " + t_->path + " version=" + lib_version_ + " gpus=" +
                 std::to_string(devs_.size()));
  ras_readers_.clear();
  ras_readers_.resize(devs_.size());  // entry i is created and used by device i's worker only
  ras_retry_.assign(devs_.size(), RasRetry{});
  return true;
}

void AmdSmiBackend::kfd_file_stats(uint64_t* open_fds, uint64_t* cached_reads) const {
  *open_fds = *cached_reads = 0;
  for (const auto& g : fast_)
    if (g) {
      *open_fds += g->kfd_fds();
      *cached_reads += g->kfd_reads_cached();
    }
}

int AmdSmiBackend::fast_path_devices() const {
  int n = 0;
  for (const auto& f : fast_) n += f != nullptr;
  return n;
}

namespace {
double na16(uint16_t x) { return x == 0xFFFF ? kNaN : x; }
double na32(uint32_t x) { return x == 0xFFFFFFFFu ? kNaN : x; }
double na64(uint64_t x) { return x == ~0ull ? kNaN : static_cast<double>(x); }
std::string fmtd(double v) {
  char b[32];
  snprintf(b, sizeof b, "%.6g", v);
  return b;
}
}  // namespace

std::vector<std::tuple<std::string, double, double>> AmdSmiBackend::compare_tables(int i, std::string* err) {
  std::vector<std::tuple<std::string, double, double>> out;
  if (i < 0 || i >= static_cast<int>(devs_.size())) {
    if (err) *err = "no such device";
    return out;
  }
  amdsmi_gpu_metrics_t a;
  if (t_->amdsmi_get_gpu_metrics_info(handles_[i], &a) != AMDSMI_STATUS_SUCCESS) {
    if (err) *err = "amdsmi_get_gpu_metrics_info failed";
    return out;
  }
  SysfsGpu own;
  SysfsGpu* g = fast_[i].get();
  std::string why;
  if (!g) {
    if (!own.open(sys_root_, proc_root_, devs_[i].bdf, kfd_ids_[i], devs_[i].drm_render, &why)) {
      if (err) *err = why;
      return out;
    }
    g = &own;
  }
  kgm::V18 k;
  if (!g->read_metrics(&k, &why)) {
    if (err) *err = why;
    return out;
  }
  amdsmi_gpu_metrics_t s;
  kgm::to_smi(k, &s);
#define CMP16(f) out.emplace_back(#f, na16(a.f), na16(s.f));
#define CMP32(f) out.emplace_back(#f, na32(a.f), na32(s.f));
#define CMP64(f) out.emplace_back(#f, na64(a.f), na64(s.f));
  out.emplace_back("structure_size", a.common_header.structure_size, s.common_header.structure_size);
  out.emplace_back("format_revision", a.common_header.format_revision, s.common_header.format_revision);
  out.emplace_back("content_revision", a.common_header.content_revision, s.common_header.content_revision);
  CMP16(temperature_edge) CMP16(temperature_hotspot) CMP16(temperature_mem) CMP16(temperature_vrgfx)
  CMP16(temperature_vrsoc) CMP16(temperature_vrmem) CMP16(average_gfx_activity) CMP16(average_umc_activity)
  CMP16(average_mm_activity) CMP16(average_socket_power) CMP16(current_socket_power)
  CMP64(energy_accumulator) CMP64(system_clock_counter) CMP64(firmware_timestamp)
  CMP16(average_gfxclk_frequency) CMP16(current_gfxclk) CMP16(current_socclk) CMP16(current_uclk)
  CMP16(current_vclk0) CMP16(current_dclk0) CMP32(throttle_status) CMP64(indep_throttle_status)
  CMP16(current_fan_speed) CMP16(pcie_link_width) CMP16(pcie_link_speed) CMP32(gfx_activity_acc)
  CMP32(mem_activity_acc) CMP16(voltage_soc) CMP16(voltage_gfx) CMP16(voltage_mem) CMP32(gfxclk_lock_status)
  CMP16(xgmi_link_width) CMP16(xgmi_link_speed) CMP64(pcie_bandwidth_acc) CMP64(pcie_bandwidth_inst)
  CMP64(pcie_l0_to_recov_count_acc) CMP64(pcie_replay_count_acc) CMP64(pcie_replay_rover_count_acc)
  CMP32(pcie_nak_sent_count_acc) CMP32(pcie_nak_rcvd_count_acc) CMP64(accumulation_counter)
  CMP64(prochot_residency_acc) CMP64(ppt_residency_acc) CMP64(socket_thm_residency_acc)
  CMP64(vr_thm_residency_acc) CMP64(hbm_thm_residency_acc) CMP16(num_partition)
  CMP32(pcie_lc_perf_other_end_recovery) CMP64(vram_max_bandwidth)
  for (int k2 = 0; k2 < AMDSMI_MAX_NUM_XGMI_LINKS; ++k2) {
    const std::string n = "[" + std::to_string(k2) + "]";
    out.emplace_back("xgmi_read_data_acc" + n, na64(a.xgmi_read_data_acc[k2]), na64(s.xgmi_read_data_acc[k2]));
    out.emplace_back("xgmi_write_data_acc" + n, na64(a.xgmi_write_data_acc[k2]), na64(s.xgmi_write_data_acc[k2]));
    out.emplace_back("xgmi_link_status" + n, na16(a.xgmi_link_status[k2]), na16(s.xgmi_link_status[k2]));
  }
  for (int k2 = 0; k2 < AMDSMI_MAX_NUM_GFX_CLKS; ++k2)
    out.emplace_back("current_gfxclks[" + std::to_string(k2) + "]", na16(a.current_gfxclks[k2]),
                     na16(s.current_gfxclks[k2]));
  for (int k2 = 0; k2 < AMDSMI_MAX_NUM_CLKS; ++k2) {
    const std::string n = "[" + std::to_string(k2) + "]";
    out.emplace_back("current_socclks" + n, na16(a.current_socclks[k2]), na16(s.current_socclks[k2]));
    out.emplace_back("current_vclk0s" + n, na16(a.current_vclk0s[k2]), na16(s.current_vclk0s[k2]));
    out.emplace_back("current_dclk0s" + n, na16(a.current_dclk0s[k2]), na16(s.current_dclk0s[k2]));
  }
  for (int x = 0; x < AMDSMI_MAX_NUM_XCP; ++x)
    for (int c = 0; c < AMDSMI_MAX_NUM_XCC; ++c) {
      const std::string n = "xcp_stats[" + std::to_string(x) + "].";
      const std::string ix = "[" + std::to_string(c) + "]";
      out.emplace_back(n + "gfx_busy_inst" + ix, na32(a.xcp_stats[x].gfx_busy_inst[c]),
                       na32(s.xcp_stats[x].gfx_busy_inst[c]));
      out.emplace_back(n + "gfx_busy_acc" + ix, na64(a.xcp_stats[x].gfx_busy_acc[c]),
                       na64(s.xcp_stats[x].gfx_busy_acc[c]));
      out.emplace_back(n + "gfx_low_utilization_acc" + ix, na64(a.xcp_stats[x].gfx_low_utilization_acc[c]),
                       na64(s.xcp_stats[x].gfx_low_utilization_acc[c]));
    }
#undef CMP16
#undef CMP32
#undef CMP64
  return out;
}

// Stable fields that must agree between libamd_smi and the sysfs decode before the fast path is
// trusted for a device (a mismatch means the kernel layout is not the one sysfs_fast.h knows).
bool AmdSmiBackend::validate_fast(int i, std::string* why) {
  std::string err;
  auto rows = compare_tables(i, &err);
  if (rows.empty()) {
    *why = "validation read failed: " + err;
    return false;
  }
  static const char* exact[] = {"format_revision", "content_revision", "pcie_link_width",
                                "xgmi_link_width", "xgmi_link_speed", "num_partition", "vram_max_bandwidth",
                                "xgmi_link_status[1]", "xgmi_link_status[7]"};
  static const char* close[] = {"temperature_hotspot", "temperature_mem", "current_uclk"};
  for (const auto& [name, a, s] : rows) {
    const bool a_na = a != a, s_na = s != s;
    for (const char* e : exact)
      if (name == e && (a_na != s_na || (!a_na && a != s))) {
        *why = "sysfs table disagrees with amdsmi on " + name + " (" + fmtd(a) + " vs " +
               fmtd(s) + ")";
        return false;
      }
    for (const char* c : close)
      if (name == c && (a_na != s_na || (!a_na && std::fabs(a - s) > std::max(5.0, 0.1 * std::fabs(a))))) {
        *why = "sysfs table disagrees with amdsmi on " + name + " (" + fmtd(a) + " vs " +
               fmtd(s) + ")";
        return false;
      }
    if (name == "firmware_timestamp" && !a_na && !s_na && (s < a || s - a > 1e10)) {
      *why = "sysfs firmware_timestamp not after amdsmi's";
      return false;
    }
  }
  return true;
}

void AmdSmiBackend::sample(int i, DeviceSample* out) {
  out->reset();
  int64_t t0 = mono_ns();
  out->host_mono_ns = t0;
  out->host_wall_ns = wall_ns();
  void* h = handles_[i];
  Caps& c = caps_[i];
  auto& v = out->v;
  bool any = false;

  // Fast path: the kernel files directly (52 us + 6 us instead of ~1.1 ms through libamd_smi).
  if (SysfsGpu* g = i < static_cast<int>(fast_.size()) ? fast_[i].get() : nullptr) {
    kgm::V18 k;
    std::string why;
    int64_t ts = mono_ns();
    bool ok = g->read_metrics(&k, &why);
    record_call(kCallMetrics, mono_ns() - ts, ok);
    if (ok) {
      amdsmi_gpu_metrics_t m;
      kgm::to_smi(k, &m);
      fill_from_gpu_metrics(m, devs_[i].partition_id, AMDSMI_MAX_NUM_XCP, devs_[i].power_limit_w,
                            energy_res_uj_, out);
      ts = mono_ns();
      double used = kNaN, total = devs_[i].vram_total_bytes;
      bool vok = g->read_vram(&used, &total);
      record_call(kCallVram, mono_ns() - ts, vok);
      if (vok) {
        v[F_VRAM_USED] = used;
        v[F_VRAM_TOTAL] = total;
      }
      double gtt = kNaN;
      if (g->read_gtt(&gtt)) v[F_GTT_USED] = gtt;
      out->ok = true;
      out->sample_ns = mono_ns() - t0;
      return;
    }
    out->errors++;
    out->last_error = why;  // fall through to libamd_smi for this tick
  }

  if (c.metrics && t_->amdsmi_get_gpu_metrics_info) {
    amdsmi_gpu_metrics_t m;
    amdsmi_status_t st = SMI_TIMED(kCallMetrics, t_->amdsmi_get_gpu_metrics_info(h, &m));
    if (st == AMDSMI_STATUS_SUCCESS) {
      any = true;
      fill_from_gpu_metrics(m, devs_[i].partition_id, AMDSMI_MAX_NUM_XCP, devs_[i].power_limit_w,
                            energy_res_uj_, out);
    } else if (st == AMDSMI_STATUS_NOT_SUPPORTED) {
      c.metrics = false;
    } else {
      out->errors++;
      out->last_error = std::string("gpu_metrics: ") + smi_status_str(st);
    }
  }
  // Fallbacks for devices without a metrics table.
  if (!c.metrics && c.activity && t_->amdsmi_get_gpu_activity) {
    amdsmi_engine_usage_t u{};
    amdsmi_status_t st = SMI_TIMED(kCallActivity, t_->amdsmi_get_gpu_activity(h, &u));
    if (st == AMDSMI_STATUS_SUCCESS) {
      any = true;
      v[F_GFX_UTIL] = u32v(u.gfx_activity);
      v[F_UMC_UTIL] = u32v(u.umc_activity);
      v[F_MM_UTIL] = u32v(u.mm_activity);
    } else if (st == AMDSMI_STATUS_NOT_SUPPORTED) {
      c.activity = false;
    } else {
      out->errors++;
      out->last_error = std::string("gpu_activity: ") + smi_status_str(st);
    }
  }
  if (!c.metrics && c.power && t_->amdsmi_get_power_info) {
    amdsmi_power_info_t p{};
    amdsmi_status_t st = SMI_TIMED(kCallPower, t_->amdsmi_get_power_info(h, &p));
    if (st == AMDSMI_STATUS_SUCCESS) {
      v[F_POWER_CUR] = u32v(p.current_socket_power);
      v[F_POWER_AVG] = u32v(p.average_socket_power);
    } else if (st == AMDSMI_STATUS_NOT_SUPPORTED) {
      c.power = false;
    }
  }
  if (c.vram && t_->amdsmi_get_gpu_vram_usage) {
    amdsmi_vram_usage_t vu{};
    amdsmi_status_t st = SMI_TIMED(kCallVram, t_->amdsmi_get_gpu_vram_usage(h, &vu));
    if (st == AMDSMI_STATUS_SUCCESS) {
      any = true;
      v[F_VRAM_USED] = static_cast<double>(vu.vram_used) * 1048576.0;
      v[F_VRAM_TOTAL] = static_cast<double>(vu.vram_total) * 1048576.0;
    } else if (st == AMDSMI_STATUS_NOT_SUPPORTED) {
      c.vram = false;
    } else {
      out->errors++;
      out->last_error = std::string("vram_usage: ") + smi_status_str(st);
    }
  }
  out->ok = any;
  out->sample_ns = mono_ns() - t0;
}

bool AmdSmiBackend::processes(int i, std::vector<ProcSample>* out) {
  out->clear();
  if (SysfsGpu* g = i < static_cast<int>(fast_.size()) ? fast_[i].get() : nullptr; g && g->have_kfd()) {
    const int64_t ts = mono_ns();
    const bool ok = g->processes(out, tick_occupancy_.load(std::memory_order_relaxed));
    record_call(kCallProcs, mono_ns() - ts, ok);
    if (ok) return true;
  }
  if (!caps_[i].procs || !t_->amdsmi_get_gpu_process_list) return false;
  auto& buf = proc_buf_[i];
  for (int attempt = 0; attempt < 3; ++attempt) {
    uint32_t cap = static_cast<uint32_t>(buf.size() / sizeof(amdsmi_proc_info_t));
    uint32_t n = cap;
    auto* list = reinterpret_cast<amdsmi_proc_info_t*>(buf.data());
    amdsmi_status_t st = SMI_TIMED(kCallProcs, t_->amdsmi_get_gpu_process_list(handles_[i], &n, list));
    if (st == AMDSMI_STATUS_OUT_OF_RESOURCES) {
      buf.resize(sizeof(amdsmi_proc_info_t) * std::max<size_t>(n + 16, cap * 2));
      continue;
    }
    if (st == AMDSMI_STATUS_NOT_SUPPORTED) {
      caps_[i].procs = false;
      return false;
    }
    if (st != AMDSMI_STATUS_SUCCESS) return false;
    out->reserve(n);
    for (uint32_t k = 0; k < n && k < cap; ++k) {
      const amdsmi_proc_info_t& p = list[k];
      ProcSample ps;
      ps.pid = p.pid;
      ps.name.assign(p.name, strnlen(p.name, sizeof p.name));
      if (ps.name == "N/A") ps.name.clear();
      ps.mem_bytes = static_cast<double>(p.mem);
      ps.vram_bytes = static_cast<double>(p.memory_usage.vram_mem);
      ps.gtt_bytes = static_cast<double>(p.memory_usage.gtt_mem);
      ps.cpu_bytes = static_cast<double>(p.memory_usage.cpu_mem);
      ps.gfx_ns = p.engine_usage.gfx;
      ps.has_gfx_ns = true;
      ps.cu_occupancy = ok32(p.cu_occupancy) ? static_cast<double>(p.cu_occupancy) : kNaN;
      out->push_back(std::move(ps));
    }
    return true;
  }
  return false;
}

void AmdSmiBackend::maintain(int i) {
  if (i >= 0 && i < static_cast<int>(fast_.size()) && fast_[i]) fast_[i]->maintain();
}

bool AmdSmiBackend::prewarm(int i) {
  if (i < 0 || i >= static_cast<int>(handles_.size())) return false;
  if (i < static_cast<int>(fast_.size()) && fast_[i]) return fast_[i]->prewarm();
  // without the fast path the tick's table read goes through libamd_smi (the same sysfs file
  // underneath): warm it the same way, result discarded
  if (!t_ || !t_->amdsmi_get_gpu_metrics_info || !caps_[i].metrics) return false;
  amdsmi_gpu_metrics_t m;
  return t_->amdsmi_get_gpu_metrics_info(handles_[i], &m) == AMDSMI_STATUS_SUCCESS;
}

bool AmdSmiBackend::supports_processes(int i) const {
  if (i < 0 || i >= static_cast<int>(caps_.size())) return false;
  const bool kfd = i < static_cast<int>(fast_.size()) && fast_[i] && fast_[i]->have_kfd();
  return kfd || (caps_[i].procs && t_ && t_->amdsmi_get_gpu_process_list);
}

bool AmdSmiBackend::supports_occupancy(int i) const {
  return i >= 0 && i < static_cast<int>(fast_.size()) && fast_[i] && fast_[i]->have_kfd();
}

void AmdSmiBackend::occupancy(int i, const std::vector<uint32_t>& pids, std::vector<double>* out) {
  if (!supports_occupancy(i)) {
    out->assign(pids.size(), kNaN);
    return;
  }
  fast_[i]->occupancy(pids, out);
}

bool AmdSmiBackend::occupancy_scan(int i, std::vector<OccRead>* out) {
  return supports_occupancy(i) && fast_[i]->occupancy_scan(out);
}

bool AmdSmiBackend::supports_links() const { return t_ && t_->amdsmi_get_link_metrics; }

void AmdSmiBackend::sample_links(int i, DeviceSample* out) {
  if (!caps_[i].links || !t_->amdsmi_get_link_metrics) return;
  amdsmi_link_metrics_t lm;
  memset(&lm, 0, sizeof lm);
  amdsmi_status_t st = SMI_TIMED(kCallLinks, t_->amdsmi_get_link_metrics(handles_[i], &lm));
  if (st == AMDSMI_STATUS_NOT_SUPPORTED) {
    caps_[i].links = false;
    return;
  }
  if (st != AMDSMI_STATUS_SUCCESS) {
    out->links_read = -1;
    return;
  }
  // Raw entries only: which gpu_metrics slot an entry describes is decided by the exporter from
  // the two sources' accumulators (xgmi_map.cpp), not by position.
  // Measured on MI355X (ROCm 7.2, profiles/r3_xgmi_link_metrics.md): num_links reads 7 while the
  // library fills 8 entries -- self (bdf all-ones) plus the 7 peers -- so trusting num_links drops
  // the last peer. Entries past num_links that the library filled (non-zero bdf / rate) count too.
  int n = std::min<int>(static_cast<int>(lm.num_links), AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK);
  while (n < AMDSMI_MAX_NUM_XGMI_LINKS && (lm.links[n].bdf.as_uint != 0 || lm.links[n].bit_rate != 0)) ++n;
  out->link_entries.clear();
  for (int k = 0; k < n; ++k) {
    const auto& s = lm.links[k];
    LinkEntry e;
    e.peer_bdf = s.bdf.as_uint == ~0ull ? "" : bdf_str(s.bdf);
    if (e.peer_bdf.rfind("ffffffffffff", 0) == 0) e.peer_bdf.clear();
    e.bit_rate_gbps = ok32(s.bit_rate) ? s.bit_rate : kNaN;
    e.max_bandwidth_gbps = ok32(s.max_bandwidth) ? s.max_bandwidth : kNaN;
    e.link_type = static_cast<int>(s.link_type);
    e.has_acc = ok64(s.read) && ok64(s.write);
    e.read_kb = e.has_acc ? s.read : 0;
    e.write_kb = e.has_acc ? s.write : 0;
    out->link_entries.push_back(std::move(e));
  }
  out->links_read = 1;
}

// RAS: the kernel's ras/ text files first (no library call, readable by a non-root exporter, every
// block the driver tracks); per-block amdsmi_get_gpu_ecc_count where the directory is absent.
void AmdSmiBackend::sample_ras(int i, DeviceSample* out, int slice, int nslices) {
  if (i < 0 || i >= static_cast<int>(devs_.size())) return;
  Caps& c = caps_[i];
  const int64_t t0 = mono_ns();
  if (c.ras_sysfs) {
    if (!ras_readers_[i]) ras_readers_[i] = std::make_unique<RasSysfsReader>(sys_root_, devs_[i].bdf);
    if (static_cast<int>(ras_retry_.size()) < static_cast<int>(devs_.size())) ras_retry_.resize(devs_.size());
    if (!ras_retry_[i].due()) return;  // backing off after a transient failure
    if (ras_readers_[i]->read(slice, nslices, &out->ras)) {
      ras_retry_[i].ok();
      // a due file that failed keeps its last value: report the call failed so a stuck file shows
      // in gpumon_backend_call_errors_total{call="ras"} instead of freezing silently
      record_call(kCallRas, mono_ns() - t0, out->ras.stale_items == 0);
      return;
    }
    if (!ras_readers_[i]->missing()) {
      // files listed but none readable this time (empty cache on the first pass): a transient
      // failure must not switch ECC monitoring off for good
      ras_retry_[i].failed();
      record_call(kCallRas, mono_ns() - t0, false);
      return;
    }
    c.ras_sysfs = false;  // no ras/ error-count files on this node: do not stat it every refresh
  }
  if (slice != 0 || !t_->amdsmi_get_gpu_ecc_count || !c.ecc_blocks) return;  // one library pass per cycle
  static const std::pair<amdsmi_gpu_block_t, const char*> kBlocks[] = {
      {AMDSMI_GPU_BLOCK_UMC, "umc"},       {AMDSMI_GPU_BLOCK_SDMA, "sdma"},
      {AMDSMI_GPU_BLOCK_GFX, "gfx"},       {AMDSMI_GPU_BLOCK_MMHUB, "mmhub"},
      {AMDSMI_GPU_BLOCK_ATHUB, "athub"},   {AMDSMI_GPU_BLOCK_PCIE_BIF, "pcie_bif"},
      {AMDSMI_GPU_BLOCK_HDP, "hdp"},       {AMDSMI_GPU_BLOCK_XGMI_WAFL, "xgmi_wafl"},
      {AMDSMI_GPU_BLOCK_DF, "df"},         {AMDSMI_GPU_BLOCK_MCA, "mca"},
      {AMDSMI_GPU_BLOCK_VCN, "vcn"},       {AMDSMI_GPU_BLOCK_JPEG, "jpeg"}};
  RasSample r;
  r.source = "amdsmi";
  bool any_err = false;
  for (const auto& b : kBlocks) {
    if (!(c.ecc_blocks & static_cast<uint64_t>(b.first))) continue;
    amdsmi_error_count_t ec;
    memset(&ec, 0, sizeof ec);
    const amdsmi_status_t st = t_->amdsmi_get_gpu_ecc_count(handles_[i], b.first, &ec);
    if (st != AMDSMI_STATUS_SUCCESS) {
      // a block that never answered has no counters on this ASIC (MI355X: 12 of 19 blocks): stop
      // asking; a block that used to answer is a real error
      if (c.ecc_seen & static_cast<uint64_t>(b.first)) any_err = true;
      else c.ecc_blocks &= ~static_cast<uint64_t>(b.first);
      continue;
    }
    c.ecc_seen |= static_cast<uint64_t>(b.first);
    RasCount rc;
    rc.block = b.second;
    rc.ue = ec.uncorrectable_count;
    rc.ce = ec.correctable_count;
    rc.de = ec.deferred_count;
    rc.has_de = true;
    r.blocks.push_back(rc);
  }
  if (t_->amdsmi_get_gpu_bad_page_info) {
    uint32_t np = 0;
    if (t_->amdsmi_get_gpu_bad_page_info(handles_[i], &np, nullptr) == AMDSMI_STATUS_SUCCESS) r.bad_pages = np;
  }
  record_call(kCallRas, mono_ns() - t0, !any_err);
  if (r.blocks.empty()) return;
  r.valid = true;
  out->ras = std::move(r);
}

}  // namespace gpumon
