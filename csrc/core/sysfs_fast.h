// Direct sysfs/KFD fast path for the per-tick device reads.
//
// Measured on MI355X (tools/probe_sysfs.py, profiles/r1_sysfs_fast_path.md): going through
// libamd_smi costs ~0.86 ms for amdsmi_get_gpu_metrics_info, ~0.23 ms for the VRAM query and
// ~0.54 ms for the process list per device, while the underlying reads cost 52 us (pread of the
// 3872-byte firmware table at /sys/bus/pci/devices/<bdf>/gpu_metrics), 6 us (mem_info_vram_used)
// and ~20 us per process (/sys/class/kfd/kfd/proc/<pid>/vram_<gpu_id>). The sampler therefore
// keeps libamd_smi for enumeration, statics, links and as the fallback, and reads the hot values
// straight from the kernel through file descriptors held open across ticks.
//
// The firmware table is the kernel's `struct gpu_metrics_v1_8` (amdgpu, MI350/MI355X): header
// {structure_size=3872, format 1, content 8}. It is decoded into the amdsmi/rsmi gpu_metrics
// structs (same field names) so the exposition path (metrics_table.h) is shared. The fast path is
// only enabled for a device after its decoded table agrees with libamd_smi's on the stable
// fields (AmdSmiBackend::init), so a layout change in a future firmware/driver disables it
// instead of exporting garbage.
#pragma once

#include <cstddef>
#include <cstdint>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "sample.h"

namespace gpumon {
namespace kgm {

constexpr int kLinks = 8, kGfxClks = 8, kClks = 4, kXcp = 8, kXcc = 8, kJpeg = 40, kVcn = 4;

struct Header {
  uint16_t structure_size;
  uint8_t format_revision;
  uint8_t content_revision;
};

struct XcpV12 {  // amdgpu_xcp_metrics_v1_2
  uint32_t gfx_busy_inst[kXcc];
  uint16_t jpeg_busy[kJpeg];
  uint16_t vcn_busy[kVcn];
  uint64_t gfx_busy_acc[kXcc];
  uint64_t gfx_below_host_limit_ppt_acc[kXcc];
  uint64_t gfx_below_host_limit_thm_acc[kXcc];
  uint64_t gfx_low_utilization_acc[kXcc];
  uint64_t gfx_below_host_limit_total_acc[kXcc];
};

struct V18 {  // gpu_metrics_v1_8 (natural alignment, as the kernel declares it)
  Header common_header;
  uint16_t temperature_hotspot;
  uint16_t temperature_mem;
  uint16_t temperature_vrsoc;
  uint16_t curr_socket_power;
  uint16_t average_gfx_activity;
  uint16_t average_umc_activity;
  uint64_t mem_max_bandwidth;
  uint64_t energy_accumulator;
  uint64_t system_clock_counter;
  uint32_t accumulation_counter;
  uint32_t prochot_residency_acc;
  uint32_t ppt_residency_acc;
  uint32_t socket_thm_residency_acc;
  uint32_t vr_thm_residency_acc;
  uint32_t hbm_thm_residency_acc;
  uint32_t gfxclk_lock_status;
  uint16_t pcie_link_width;
  uint16_t pcie_link_speed;
  uint16_t xgmi_link_width;
  uint16_t xgmi_link_speed;
  uint32_t gfx_activity_acc;
  uint32_t mem_activity_acc;
  uint64_t pcie_bandwidth_acc;
  uint64_t pcie_bandwidth_inst;
  uint64_t pcie_l0_to_recov_count_acc;
  uint64_t pcie_replay_count_acc;
  uint64_t pcie_replay_rover_count_acc;
  uint32_t pcie_nak_sent_count_acc;
  uint32_t pcie_nak_rcvd_count_acc;
  uint64_t xgmi_read_data_acc[kLinks];
  uint64_t xgmi_write_data_acc[kLinks];
  uint16_t xgmi_link_status[kLinks];
  uint16_t padding;
  uint64_t firmware_timestamp;
  uint16_t current_gfxclk[kGfxClks];
  uint16_t current_socclk[kClks];
  uint16_t current_vclk0[kClks];
  uint16_t current_dclk0[kClks];
  uint16_t current_uclk;
  uint16_t num_partition;
  XcpV12 xcp_stats[kXcp];
  uint32_t pcie_lc_perf_other_end_recovery;
};

static_assert(sizeof(XcpV12) == 440, "xcp_metrics_v1_2 layout");
static_assert(offsetof(V18, xgmi_read_data_acc) == 136, "gpu_metrics_v1_8 layout");
static_assert(offsetof(V18, firmware_timestamp) == 288, "gpu_metrics_v1_8 layout");
static_assert(offsetof(V18, xcp_stats) == 344, "gpu_metrics_v1_8 layout");
static_assert(sizeof(V18) == 3872, "gpu_metrics_v1_8 is 3872 bytes on MI355X");

inline uint64_t w32(uint32_t x) { return x == 0xFFFFFFFFu ? ~0ull : x; }

// Kernel v1.8 table -> amdsmi_gpu_metrics_t / rsmi_gpu_metrics_t (identical field names).
// Fields the v1.8 table does not carry stay all-ones (= N/A, the firmware convention).
template <typename M>
void to_smi(const V18& k, M* m) {
  memset(m, 0xFF, sizeof *m);
  m->common_header.structure_size = k.common_header.structure_size;
  m->common_header.format_revision = k.common_header.format_revision;
  m->common_header.content_revision = k.common_header.content_revision;
  m->temperature_hotspot = k.temperature_hotspot;
  m->temperature_mem = k.temperature_mem;
  m->temperature_vrsoc = k.temperature_vrsoc;
  m->current_socket_power = k.curr_socket_power;
  m->average_gfx_activity = k.average_gfx_activity;
  m->average_umc_activity = k.average_umc_activity;
  m->vram_max_bandwidth = k.mem_max_bandwidth;
  m->energy_accumulator = k.energy_accumulator;
  m->system_clock_counter = k.system_clock_counter;
  m->accumulation_counter = w32(k.accumulation_counter);
  m->prochot_residency_acc = w32(k.prochot_residency_acc);
  m->ppt_residency_acc = w32(k.ppt_residency_acc);
  m->socket_thm_residency_acc = w32(k.socket_thm_residency_acc);
  m->vr_thm_residency_acc = w32(k.vr_thm_residency_acc);
  m->hbm_thm_residency_acc = w32(k.hbm_thm_residency_acc);
  m->gfxclk_lock_status = k.gfxclk_lock_status;
  m->pcie_link_width = k.pcie_link_width;
  m->pcie_link_speed = k.pcie_link_speed;
  m->xgmi_link_width = k.xgmi_link_width;
  m->xgmi_link_speed = k.xgmi_link_speed;
  m->gfx_activity_acc = k.gfx_activity_acc;
  m->mem_activity_acc = k.mem_activity_acc;
  m->pcie_bandwidth_acc = k.pcie_bandwidth_acc;
  m->pcie_bandwidth_inst = k.pcie_bandwidth_inst;
  m->pcie_l0_to_recov_count_acc = k.pcie_l0_to_recov_count_acc;
  m->pcie_replay_count_acc = k.pcie_replay_count_acc;
  m->pcie_replay_rover_count_acc = k.pcie_replay_rover_count_acc;
  m->pcie_nak_sent_count_acc = k.pcie_nak_sent_count_acc;
  m->pcie_nak_rcvd_count_acc = k.pcie_nak_rcvd_count_acc;
  for (int i = 0; i < kLinks; ++i) {
    m->xgmi_read_data_acc[i] = k.xgmi_read_data_acc[i];
    m->xgmi_write_data_acc[i] = k.xgmi_write_data_acc[i];
    m->xgmi_link_status[i] = k.xgmi_link_status[i];
  }
  m->firmware_timestamp = k.firmware_timestamp;
  for (int i = 0; i < kGfxClks; ++i) m->current_gfxclks[i] = k.current_gfxclk[i];
  for (int i = 0; i < kClks; ++i) {
    m->current_socclks[i] = k.current_socclk[i];
    m->current_vclk0s[i] = k.current_vclk0[i];
    m->current_dclk0s[i] = k.current_dclk0[i];
  }
  m->current_gfxclk = k.current_gfxclk[0];
  m->current_socclk = k.current_socclk[0];
  m->current_vclk0 = k.current_vclk0[0];
  m->current_dclk0 = k.current_dclk0[0];
  m->current_uclk = k.current_uclk;
  m->num_partition = k.num_partition;
  for (int x = 0; x < kXcp; ++x) {
    const XcpV12& s = k.xcp_stats[x];
    auto& d = m->xcp_stats[x];
    for (int i = 0; i < kXcc; ++i) {
      d.gfx_busy_inst[i] = s.gfx_busy_inst[i];
      d.gfx_busy_acc[i] = s.gfx_busy_acc[i];
      d.gfx_below_host_limit_ppt_acc[i] = s.gfx_below_host_limit_ppt_acc[i];
      d.gfx_below_host_limit_thm_acc[i] = s.gfx_below_host_limit_thm_acc[i];
      d.gfx_low_utilization_acc[i] = s.gfx_low_utilization_acc[i];
      d.gfx_below_host_limit_total_acc[i] = s.gfx_below_host_limit_total_acc[i];
    }
    for (int i = 0; i < kJpeg; ++i) d.jpeg_busy[i] = s.jpeg_busy[i];
    for (int i = 0; i < kVcn; ++i) d.vcn_busy[i] = s.vcn_busy[i];
  }
  m->pcie_lc_perf_other_end_recovery = k.pcie_lc_perf_other_end_recovery;
}

}  // namespace kgm

// One device's kernel files, opened once and re-read with pread(…, 0) every tick.
class SysfsGpu {
 public:
  SysfsGpu() = default;
  ~SysfsGpu();
  SysfsGpu(const SysfsGpu&) = delete;
  SysfsGpu& operator=(const SysfsGpu&) = delete;

  // sys_root: "/sys" (tests point it at a fake tree); proc_root: "/proc".
  bool open(const std::string& sys_root, const std::string& proc_root, const std::string& bdf,
            uint64_t kfd_gpu_id, int drm_render, std::string* why);
  // Raw firmware table; false if the read failed or it is not a v1.8 table.
  bool read_metrics(kgm::V18* out, std::string* why);
  bool read_vram(double* used_bytes, double* total_bytes);
  bool read_gtt(double* used_bytes);
  // Compute processes with memory on this GPU (KFD), plus DRM fdinfo gfx engine time / memory.
  // read_occupancy false: leave cu_occupancy NaN (the device worker sub-samples it between ticks,
  // and the KFD read is the costliest per-process file: it walks the process's queues).
  bool processes(std::vector<ProcSample>* out, bool read_occupancy = true);
  // Instantaneous KFD cu_occupancy of each pid on this GPU (NaN where the file is unreadable).
  void occupancy(const std::vector<uint32_t>& pids, std::vector<double>* out);
  // Every KFD process on this GPU with its cu_occupancy and VRAM (no fdinfo): the between-ticks
  // sub-sample, which also sees processes started since the last tick.
  bool occupancy_scan(std::vector<OccRead>* out);
  bool have_kfd() const { return kfd_gpu_id_ != 0; }
  // Off-tick upkeep (device worker, after it published): refreshes due /proc/<pid>/fd scans.
  void maintain();
  // One gpu_metrics read whose table is discarded: leaves the SMU's fetch path warm for the tick.
  bool prewarm();
  // KFD per-pid files held open right now, and reads served from a kept fd (tests / self-metrics).
  size_t kfd_fds();
  uint64_t kfd_reads_cached() const { return kfd_reads_cached_.load(std::memory_order_relaxed); }

 private:
  void fdinfo_usage(uint32_t pid, ProcSample* p);
  // Hardware queues `pid` holds on this GPU: proc/<pid>/queues/<qid>/gpuid == this GPU's KFD id
  // (-1: the directory is unreadable), from the node-wide KfdQueueTables.
  int queues_here(uint32_t pid, int64_t now);
  // /sys/class/kfd/kfd/proc is not namespaced: it lists every KFD process of the host, on every
  // GPU (15-17 on a shared MI355X box, 1 of them on the container's GPU). A process found not to
  // be on this GPU is not asked again for kNotHereNs (each ask is an open() that fails, ~4-6 us):
  // a process that starts using this GPU later is picked up within that time. Pids that left the
  // listing are dropped. Shared by the tick's process list and the between-tick scans.
  static constexpr int64_t kNotHereNs = 1'000'000'000;
  bool skip_not_here(uint32_t pid, int64_t now);
  void note_not_here(uint32_t pid, int64_t now);
  void prune_not_here(const std::vector<uint32_t>& listed_sorted);
  std::mutex not_here_mu_;
  std::unordered_map<uint32_t, int64_t> not_here_;  // pid -> ask again after (mono ns)
  // Per-pid KFD files (vram_<gpu>, stats_<gpu>/cu_occupancy) kept open and re-read with pread(0):
  // a sub-sample costs one pread instead of open + pread + close, each open a 6-level kernfs path
  // walk (20 cu_occupancy reads per process per tick on the device worker). A read that fails on a
  // kept fd (the process exited: ENODEV; the pid was reused) reopens the path once; the files of
  // pids that left the KFD listing are closed at the next process list. At most kMaxKfdFds per GPU
  // (32 processes' pairs): past that, reads open and close as before.
  enum class KfdFile : uint8_t { kVram = 0, kOccupancy = 1 };
  bool read_kfd(uint32_t pid, KfdFile kind, char* b, size_t cap, size_t* n);
  void retain_kfd(const std::vector<uint32_t>& listed_sorted);
  static constexpr size_t kMaxKfdFds = 64;
  std::mutex kfd_fds_mu_;
  std::unordered_map<uint64_t, int> kfd_fds_;  // (pid << 1 | kind) -> fd
  std::atomic<uint64_t> kfd_reads_cached_{0};
  std::string sys_root_, proc_root_, dev_dir_;
  uint64_t kfd_gpu_id_ = 0;
  std::string render_path_;  // "/dev/dri/renderD<minor>"
  int fd_metrics_ = -1, fd_vram_used_ = -1, fd_vram_total_ = -1, fd_gtt_used_ = -1;
};

// Node-wide DRM fd tables of GPU processes. /proc/<pid>/fd lists every open file of a process
// (thousands for a data-loading trainer), so readdir + readlink over it is the one per-process read
// whose cost grows with the workload. One scan serves every GPU (each keeps the fds that point at
// its own render node); a process is scanned on the tick it first appears, and the 10 s refreshes
// (or the rescan after an fd vanished) run off the tick from SysfsGpu::maintain().
class DrmFdTables {
 public:
  static DrmFdTables& get();
  // fds of the process (pdir = <proc_root>/<pid>) that point at `render`
  void fds_for(const std::string& pdir, const std::string& render, std::vector<int>* out);
  void invalidate(const std::string& pdir);  // an fd vanished: rescan at the next maintain()
  int refresh_due(int max_scans);            // scans done
  // Drop the tables of processes under `proc_root` that are no longer in the node's KFD process
  // list (`kfd_pids`, sorted): a reused pid must not be read at the old process's fd numbers.
  void retain(const std::string& proc_root, const std::vector<uint32_t>& kfd_pids);
  void clear();  // drop every entry not being scanned right now
  uint64_t scans() const { return scans_.load(); }
  uint32_t scans_of(const std::string& pdir);  // 0 when not cached
  size_t size();

 private:
  struct Entry {
    int64_t scanned_ns = 0, used_ns = 0;
    bool want = false;
    bool scanning = false;  // first scan in flight (fds_for waits for it)
    uint32_t scans = 0;     // scans of this entry (tests: counts unaffected by other processes' entries)
    std::vector<std::pair<int, std::string>> fds;  // (fd, /dev/dri/... target)
  };
  static void scan(const std::string& pdir, std::vector<std::pair<int, std::string>>* fds);
  std::mutex mu_;
  std::condition_variable cv_;
  std::unordered_map<std::string, Entry> m_;
  std::atomic<uint64_t> scans_{0};
};

// Node-wide KFD queue lists. A process's hardware queues are listed once for every GPU
// (proc/<pid>/queues/<qid>/gpuid names each queue's GPU), so one directory scan per process per
// kRescanNs serves all device workers: on 8 GPUs, 8x fewer scans than one per (process, GPU). A
// queue created since a scan is seen within kRescanNs (its waves show in the occupancy reads
// first); processes that left the KFD listing are dropped (retain).
class KfdQueueTables {
 public:
  static constexpr int64_t kRescanNs = 2'000'000'000;
  static KfdQueueTables& get();
  // queues `pid` holds on the GPU whose KFD id is `gpu_id`; -1 = its queue list is unreadable.
  // `kfd_proc` = <sys_root>/class/kfd/kfd/proc.
  int count(const std::string& kfd_proc, uint32_t pid, uint64_t gpu_id, int64_t now);
  void retain(const std::string& kfd_proc, const std::vector<uint32_t>& listed_sorted);
  uint64_t scans() const { return scans_.load(); }
  uint32_t scans_of(const std::string& kfd_proc, uint32_t pid);  // tests
  void clear();  // tests: forget every cached list

 private:
  struct Entry {
    int64_t scanned_ns = 0;
    bool readable = false;
    uint32_t scans = 0;
    std::vector<std::pair<uint64_t, int>> per_gpu;  // (KFD gpu id, queues)
  };
  static bool scan(const std::string& qdir, std::vector<std::pair<uint64_t, int>>* per_gpu);
  std::mutex mu_;
  std::unordered_map<std::string, std::unordered_map<uint32_t, Entry>> m_;  // kfd_proc -> pid -> entry
  std::atomic<uint64_t> scans_{0};
};

}  // namespace gpumon
