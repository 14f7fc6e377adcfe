// RocmSmiBackend: fallback device backend over rocm_smi_lib (librocm_smi64), dlopen'ed through its
// own function table exactly like libamd_smi ("the rocm_smi_lib fallback sits behind
// the same dlopen table"). Used when libamd_smi is absent or fails to initialise on a host
// (`--backend auto`), or explicitly with `--backend rocm_smi`.
//
// Same firmware table (rsmi_dev_gpu_metrics_info_get -> rsmi_gpu_metrics_t, identical field names)
// converted by the shared template in metrics_table.h; VRAM via rsmi_dev_memory_*; processes via
// rsmi_compute_process_info_get + rsmi_compute_process_info_by_device_get. rocm_smi has no
// per-link metrics call: link max bandwidth comes from the table's xGMI speed x width.
#include <dlfcn.h>
#include <rocm_smi/rocm_smi.h>

#include <algorithm>
#include <cstring>

#include "backend.h"
#include "common.h"
#include "metrics_table.h"
#include "ras.h"

namespace gpumon {

#define GPUMON_RSMI_FNS(X)                  \
  X(rsmi_init)                              \
  X(rsmi_shut_down)                         \
  X(rsmi_num_monitor_devices)               \
  X(rsmi_version_get)                       \
  X(rsmi_dev_gpu_metrics_info_get)          \
  X(rsmi_dev_memory_total_get)              \
  X(rsmi_dev_memory_usage_get)              \
  X(rsmi_dev_pci_id_get)                    \
  X(rsmi_dev_unique_id_get)                 \
  X(rsmi_dev_name_get)                      \
  X(rsmi_dev_serial_number_get)             \
  X(rsmi_dev_busy_percent_get)              \
  X(rsmi_dev_memory_busy_percent_get)       \
  X(rsmi_dev_energy_count_get)              \
  X(rsmi_dev_power_cap_get)                 \
  X(rsmi_dev_compute_partition_get)         \
  X(rsmi_dev_memory_partition_get)          \
  X(rsmi_dev_partition_id_get)              \
  X(rsmi_compute_process_info_get)          \
  X(rsmi_compute_process_info_by_device_get)

struct RsmiTable {
  void* dl = nullptr;
  std::string path;
#define GPUMON_DECL(fn) decltype(&::fn) fn = nullptr;
  GPUMON_RSMI_FNS(GPUMON_DECL)
#undef GPUMON_DECL
  bool load(const std::string& explicit_path, std::string* err) {
    std::vector<std::string> c;
    if (!explicit_path.empty()) c.push_back(explicit_path);
    if (const char* e = getenv("GPUMON_ROCM_SMI_LIB")) c.emplace_back(e);
    c.emplace_back("librocm_smi64.so.1");
    c.emplace_back("librocm_smi64.so");
    c.emplace_back("/opt/rocm/lib/librocm_smi64.so.1");
    std::string errs;
    for (const auto& p : c) {
      dl = dlopen(p.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (dl) {
        path = p;
        break;
      }
      const char* e = dlerror();
      errs += p + ": " + (e ? e : "?") + "; ";
    }
    if (!dl) {
      *err = "cannot dlopen librocm_smi64 (" + errs + ")";
      return false;
    }
#define GPUMON_SYM(fn) fn = reinterpret_cast<decltype(fn)>(dlsym(dl, #fn));
    GPUMON_RSMI_FNS(GPUMON_SYM)
#undef GPUMON_SYM
    if (!rsmi_init || !rsmi_num_monitor_devices || !rsmi_shut_down) {
      *err = "librocm_smi64 lacks rsmi_init/rsmi_num_monitor_devices";
      dlclose(dl);
      dl = nullptr;
      return false;
    }
    return true;
  }
  ~RsmiTable() {
    if (dl) dlclose(dl);
  }
};

#define RSMI_TIMED(call_id, expr)                                                       \
  ([&]() {                                                                              \
    const int64_t t_start_ = mono_ns();                                                 \
    const rsmi_status_t s_ = (expr);                                                    \
    record_call(call_id, mono_ns() - t_start_,                                          \
                s_ == RSMI_STATUS_SUCCESS || s_ == RSMI_STATUS_NOT_SUPPORTED ||          \
                    s_ == RSMI_STATUS_INSUFFICIENT_SIZE);                               \
    return s_;                                                                          \
  }())

RocmSmiBackend::RocmSmiBackend(std::string lib_path) : lib_path_(std::move(lib_path)) {}
RocmSmiBackend::~RocmSmiBackend() { shutdown(); }

void RocmSmiBackend::shutdown() {
  if (t_ && inited_) t_->rsmi_shut_down();
  inited_ = false;
  devs_.clear();
  idx_.clear();
}

bool RocmSmiBackend::init(std::string* err) {
  shutdown();
  if (!t_) t_ = std::make_unique<RsmiTable>();
  if (!t_->dl && !t_->load(lib_path_, err)) return false;
  rsmi_status_t st = t_->rsmi_init(0);
  if (st != RSMI_STATUS_SUCCESS) {
    *err = "rsmi_init failed (" + std::to_string(static_cast<int>(st)) + ")";
    return false;
  }
  inited_ = true;
  if (t_->rsmi_version_get) {
    rsmi_version_t v{};
    if (t_->rsmi_version_get(&v) == RSMI_STATUS_SUCCESS)
      lib_version_ = std::to_string(v.major) + "." + std::to_string(v.minor) + "." + std::to_string(v.patch);
  }
  uint32_t n = 0;
  t_->rsmi_num_monitor_devices(&n);
  for (uint32_t i = 0; i < n; ++i) {
    char buf[256] = {0};
    uint64_t bdf = 0;
    std::string bdf_s;
    if (t_->rsmi_dev_pci_id_get && t_->rsmi_dev_pci_id_get(i, &bdf) == RSMI_STATUS_SUCCESS) {
      // rsmi BDFID: domain[63:32] bus[15:8] device[7:3] function[2:0]
      snprintf(buf, sizeof buf, "%04llx:%02llx:%02llx.%llx", static_cast<unsigned long long>(bdf >> 32),
               static_cast<unsigned long long>((bdf >> 8) & 0xFF), static_cast<unsigned long long>((bdf >> 3) & 0x1F),
               static_cast<unsigned long long>(bdf & 0x7));
      bdf_s = buf;
    }
    // rsmi's index is the hip_id: its enumeration follows the KFD node order, as HIP's does
    if (!keep(static_cast<int>(i), bdf_s)) continue;
    DeviceStatic d;
    d.index = static_cast<int>(devs_.size());
    d.hip_id = static_cast<int>(i);
    d.gpu_id = std::to_string(i);
    d.bdf = bdf_s;
    memset(buf, 0, sizeof buf);
    if (t_->rsmi_dev_name_get && t_->rsmi_dev_name_get(i, buf, sizeof buf) == RSMI_STATUS_SUCCESS) d.model = buf;
    memset(buf, 0, sizeof buf);
    if (t_->rsmi_dev_serial_number_get && t_->rsmi_dev_serial_number_get(i, buf, sizeof buf) == RSMI_STATUS_SUCCESS)
      d.serial = buf;
    uint64_t uid = 0;
    if (t_->rsmi_dev_unique_id_get && t_->rsmi_dev_unique_id_get(i, &uid) == RSMI_STATUS_SUCCESS) {
      snprintf(buf, sizeof buf, "%016llx", static_cast<unsigned long long>(uid));
      d.uuid = buf;
    }
    memset(buf, 0, sizeof buf);
    if (t_->rsmi_dev_compute_partition_get &&
        t_->rsmi_dev_compute_partition_get(i, buf, sizeof buf) == RSMI_STATUS_SUCCESS)
      d.compute_partition = buf;
    memset(buf, 0, sizeof buf);
    if (t_->rsmi_dev_memory_partition_get &&
        t_->rsmi_dev_memory_partition_get(i, buf, sizeof buf) == RSMI_STATUS_SUCCESS)
      d.memory_partition = buf;
    uint32_t pid = 0;
    if (t_->rsmi_dev_partition_id_get && t_->rsmi_dev_partition_id_get(i, &pid) == RSMI_STATUS_SUCCESS)
      d.partition_id = static_cast<int>(pid);
    uint64_t cap = 0;
    if (t_->rsmi_dev_power_cap_get && t_->rsmi_dev_power_cap_get(i, 0, &cap) == RSMI_STATUS_SUCCESS)
      d.power_limit_w = static_cast<double>(cap) * 1e-6;  // microwatts
    uint64_t tot = 0;
    if (t_->rsmi_dev_memory_total_get && t_->rsmi_dev_memory_total_get(i, RSMI_MEM_TYPE_VRAM, &tot) == RSMI_STATUS_SUCCESS)
      d.vram_total_bytes = static_cast<double>(tot);
    d.gfx_target = "gfx950";
    devs_.push_back(std::move(d));
    idx_.push_back(i);
  }
  if (devs_.empty()) {
    *err = "rocm_smi: no GPUs found (after device filter)";
    return false;
  }
  if (t_->rsmi_dev_energy_count_get) {
    uint64_t e = 0, ts = 0;
    float res = 0;
    if (t_->rsmi_dev_energy_count_get(idx_[0], &e, &res, &ts) == RSMI_STATUS_SUCCESS && res > 0) energy_res_uj_ = res;
  }
  GPUMON_LOG(LogLevel::kInfo, "rocm_smi",
             "loaded " + t_->path + " version=" + lib_version_ + " gpus=" + std::to_string(devs_.size()));
  ras_readers_.clear();
  ras_readers_.resize(devs_.size());
  ras_retry_.assign(devs_.size(), RasRetry{});
  ras_missing_.assign(devs_.size(), 0);
  return true;
}

void RocmSmiBackend::sample(int i, DeviceSample* out) {
  out->reset();
  const int64_t t0 = mono_ns();
  out->host_mono_ns = t0;
  out->host_wall_ns = wall_ns();
  const uint32_t dv = idx_[i];
  bool any = false;
  if (metrics_ok_ && t_->rsmi_dev_gpu_metrics_info_get) {
    rsmi_gpu_metrics_t m;
    rsmi_status_t st = RSMI_TIMED(kCallMetrics, t_->rsmi_dev_gpu_metrics_info_get(dv, &m));
    if (st == RSMI_STATUS_SUCCESS) {
      any = true;
      fill_from_gpu_metrics(m, devs_[i].partition_id, RSMI_MAX_NUM_XCP, devs_[i].power_limit_w, energy_res_uj_, out);
    } else if (st == RSMI_STATUS_NOT_SUPPORTED) {
      metrics_ok_ = false;
    } else {
      out->errors++;
      out->last_error = "rsmi_dev_gpu_metrics_info_get: " + std::to_string(static_cast<int>(st));
    }
  }
  if (!metrics_ok_) {
    uint32_t busy = 0, mbusy = 0;
    if (t_->rsmi_dev_busy_percent_get &&
        RSMI_TIMED(kCallActivity, t_->rsmi_dev_busy_percent_get(dv, &busy)) == RSMI_STATUS_SUCCESS) {
      any = true;
      out->v[F_GFX_UTIL] = busy;
    }
    if (t_->rsmi_dev_memory_busy_percent_get && t_->rsmi_dev_memory_busy_percent_get(dv, &mbusy) == RSMI_STATUS_SUCCESS)
      out->v[F_UMC_UTIL] = mbusy;
  }
  uint64_t used = 0, tot = 0;
  if (t_->rsmi_dev_memory_usage_get &&
      RSMI_TIMED(kCallVram, t_->rsmi_dev_memory_usage_get(dv, RSMI_MEM_TYPE_VRAM, &used)) == RSMI_STATUS_SUCCESS) {
    any = true;
    out->v[F_VRAM_USED] = static_cast<double>(used);
    out->v[F_VRAM_TOTAL] = devs_[i].vram_total_bytes;
    if (!has(out->v[F_VRAM_TOTAL]) && t_->rsmi_dev_memory_total_get &&
        t_->rsmi_dev_memory_total_get(dv, RSMI_MEM_TYPE_VRAM, &tot) == RSMI_STATUS_SUCCESS)
      out->v[F_VRAM_TOTAL] = static_cast<double>(tot);
  }
  out->ok = any;
  out->sample_ns = mono_ns() - t0;
}

bool RocmSmiBackend::supports_processes(int) const {
  return t_ && t_->rsmi_compute_process_info_get && t_->rsmi_compute_process_info_by_device_get;
}

bool RocmSmiBackend::processes(int i, std::vector<ProcSample>* out) {
  out->clear();
  if (!t_->rsmi_compute_process_info_get || !t_->rsmi_compute_process_info_by_device_get) return false;
  const int64_t t0 = mono_ns();
  std::vector<rsmi_process_info_t> all(64);
  uint32_t n = static_cast<uint32_t>(all.size());
  rsmi_status_t st = t_->rsmi_compute_process_info_get(all.data(), &n);
  if (st == RSMI_STATUS_INSUFFICIENT_SIZE || n > all.size()) {
    all.resize(n + 16);
    n = static_cast<uint32_t>(all.size());
    st = t_->rsmi_compute_process_info_get(all.data(), &n);
  }
  if (st != RSMI_STATUS_SUCCESS) {
    record_call(kCallProcs, mono_ns() - t0, false);
    return false;
  }
  for (uint32_t k = 0; k < n && k < all.size(); ++k) {
    rsmi_process_info_t pi{};
    if (t_->rsmi_compute_process_info_by_device_get(all[k].process_id, idx_[i], &pi) != RSMI_STATUS_SUCCESS) continue;
    // rocm_smi_lib answers SUCCESS for node-wide KFD processes that hold nothing on this GPU
    // (seen on MI355X: 8 rows where libamd_smi lists 2); keep only those with memory here.
    if (pi.vram_usage == 0) continue;
    ProcSample p;
    p.pid = pi.process_id;
    p.vram_bytes = static_cast<double>(pi.vram_usage);
    p.mem_bytes = p.vram_bytes;
    p.cu_occupancy = pi.cu_occupancy == CU_OCCUPANCY_INVALID ? kNaN : static_cast<double>(pi.cu_occupancy);
    out->push_back(std::move(p));
  }
  record_call(kCallProcs, mono_ns() - t0, true);
  return true;
}

void RocmSmiBackend::sample_ras(int i, DeviceSample* out, int slice, int nslices) {
  if (i < 0 || i >= static_cast<int>(devs_.size())) return;
  if (i < static_cast<int>(ras_missing_.size()) && ras_missing_[i]) return;  // no ras/ files on this node
  if (!ras_readers_[i]) ras_readers_[i] = std::make_unique<RasSysfsReader>(sys_root_, devs_[i].bdf);
  if (static_cast<int>(ras_retry_.size()) < static_cast<int>(devs_.size())) ras_retry_.resize(devs_.size());
  if (!ras_retry_[i].due()) return;  // backing off after a transient failure
  const int64_t t0 = mono_ns();
  const bool ok = ras_readers_[i]->read(slice, nslices, &out->ras);
  if (ok) {
    ras_retry_[i].ok();
  } else if (ras_readers_[i]->missing()) {
    // no error-count files (VM guest, RAS disabled): stop re-listing the directory every tick
    if (i < static_cast<int>(ras_missing_.size())) ras_missing_[i] = 1;
  } else {
    ras_retry_[i].failed();  // files listed but none readable this time: retry with backoff
  }
  record_call(kCallRas, mono_ns() - t0, ok && out->ras.stale_items == 0);
}

}  // namespace gpumon
