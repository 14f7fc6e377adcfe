// Device backends: where samples come from.
//
// Reference equivalent: the nvidia-smi CLI subprocesses (/root/reference/gpu.py:104-116) behind
// the commandexists() probe (gpu.py:28-33,260). Here a backend is an in-process C++ object:
//   - AmdSmiBackend: libamd_smi resolved at run time through SmiTable (dlopen; the role the
//     vendored libltdl.so.7 played for the reference's docker CLI).
//   - MockBackend:   N scripted fake GPUs for CPU tests, benches and fault injection.
#pragma once

#include <atomic>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "common.h"
#include "ras.h"
#include "sample.h"

namespace gpumon {

class Backend {
 public:
  virtual ~Backend() = default;
  virtual std::string name() const = 0;
  // (Re)initialise; returns false with *err set if the device layer is unavailable.
  virtual bool init(std::string* err) = 0;
  virtual void shutdown() {}
  virtual int device_count() const = 0;
  virtual const DeviceStatic& static_info(int i) const = 0;
  // Fill one device sample. Must not throw; failures are reported in out->ok / errors.
  virtual void sample(int i, DeviceSample* out) = 0;
  // GPU processes on device i. Returns false if the call failed.
  virtual bool processes(int i, std::vector<ProcSample>* out) = 0;
  // Can device i list processes at all? A false processes() on a device that can is a failure
  // (counted, and the last good list is held for a few ticks); on one that cannot, it is not.
  virtual bool supports_processes(int /*i*/) const { return true; }
  // Optional: per-link metrics are expensive (~1 ms); sampled every `link_every` ticks.
  virtual bool supports_links() const { return false; }
  virtual void sample_links(int, DeviceSample*) {}
  // Optional: RAS / ECC counters (ras.h) into out->ras. Called on the ticks where a RAS slice is due
  // (Exporter::sample_devices: `ras_slices` consecutive ticks out of every `ras_every`) with slice
  // in [0, nslices), nslices = `ras_slices`: a source that can refresh part of its counters (the
  // sysfs files) reads that slice; others refresh everything on slice 0 only.
  virtual bool supports_ras() const { return false; }
  // Optional: instantaneous KFD cu_occupancy of `pids` on device i (out[k] NaN = unreadable).
  // Cheap (~27 us per process on MI355X): the device worker sub-samples it between ticks.
  virtual bool supports_occupancy(int /*i*/) const { return false; }
  virtual void occupancy(int, const std::vector<uint32_t>& pids, std::vector<double>* out) {
    out->assign(pids.size(), kNaN);
  }
  // Optional: cu_occupancy + VRAM of EVERY process on device i right now, newly started ones
  // included (the device worker's sub-samples; false = unsupported, use occupancy() on the pids of
  // the last tick instead).
  virtual bool occupancy_scan(int, std::vector<OccRead>*) { return false; }
  virtual void sample_ras(int, DeviceSample*, int /*slice*/ = 0, int /*nslices*/ = 1) {}
  // The device workers sub-sample cu_occupancy between ticks (occupancy_scan / occupancy): the
  // process list at the tick may then skip its own occupancy read (cu_occupancy left NaN).
  virtual void set_tick_occupancy(bool /*on*/) {}
  // May processes(i) run on another thread while sample(i) runs (the device worker then overlaps
  // the process list with the firmware-table read)? Only where both read independent files.
  virtual bool concurrent_processes(int /*i*/) const { return false; }
  // Upkeep that must stay off the tick's critical path (the device worker calls it after it
  // published the tick's sample): e.g. refreshing cached /proc fd tables.
  virtual void maintain(int /*i*/) {}
  // Wake the device's firmware-table path a few ms before a tick (the device worker calls it at
  // deadline - prewarm_ms): on MI355X a gpu_metrics fetch costs ~50 us when the SMU served one
  // within ~5 ms and 150-300 us after a longer gap; spinning the CPU instead does not help
  // (profiles/r3_capacity.md). Returns false where the backend has nothing to warm.
  virtual bool prewarm(int /*i*/) { return false; }
  // Restrict to a subset of devices (empty = all). Applied at init(). An entry is a hip_id ("3")
  // or a PCI BDF ("0000:75:00.0", domain optional): a process that sees its GPUs through
  // HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES numbers them 0..n-1, while libamd_smi's hip_id is
  // the node-wide index, so callers that loaded HIP ordinals name them by BDF
  // (hipDeviceGetPCIBusId, gpumon/parallel/devmap.py). Unparseable entries match nothing.
  void set_device_filter(const std::vector<std::string>& ids) {
    filter_ids_.clear();
    filter_bdfs_.clear();
    for (const auto& s : ids) {
      std::string b = normalize_bdf(s);
      if (!b.empty()) {
        filter_bdfs_.push_back(b);
        continue;
      }
      char* end = nullptr;
      long v = strtol(s.c_str(), &end, 10);
      filter_ids_.push_back(end && end != s.c_str() && *end == 0 && v >= 0 ? static_cast<int>(v) : -1);
    }
  }
  bool has_device_filter() const { return !filter_ids_.empty() || !filter_bdfs_.empty(); }

  // Per-call latency accounting (exported as gpumon_backend_call_* self-metrics).
  enum Call { kCallMetrics = 0, kCallVram, kCallProcs, kCallLinks, kCallActivity, kCallPower, kCallRas, kCallCount };
  static const char* call_name(int c) {
    static const char* n[] = {"gpu_metrics", "vram_usage", "process_list", "link_metrics", "gpu_activity",
                              "power_info", "ras"};
    return c >= 0 && c < kCallCount ? n[c] : "?";
  }
  struct CallSnap {
    std::string call;
    uint64_t n = 0, errors = 0;
    double seconds = 0;
  };
  std::vector<CallSnap> call_stats() const {
    std::vector<CallSnap> v;
    for (int c = 0; c < kCallCount; ++c) {
      uint64_t n = calls_n_[c].load(std::memory_order_relaxed);
      if (!n) continue;
      v.push_back({call_name(c), n, calls_err_[c].load(std::memory_order_relaxed),
                   calls_ns_[c].load(std::memory_order_relaxed) * 1e-9});
    }
    return v;
  }

 protected:
  void record_call(int c, int64_t ns, bool ok) {
    calls_n_[c].fetch_add(1, std::memory_order_relaxed);
    calls_ns_[c].fetch_add(static_cast<uint64_t>(ns > 0 ? ns : 0), std::memory_order_relaxed);
    if (!ok) calls_err_[c].fetch_add(1, std::memory_order_relaxed);
  }
  std::atomic<uint64_t> calls_n_[kCallCount] = {};
  std::atomic<uint64_t> calls_ns_[kCallCount] = {};
  std::atomic<uint64_t> calls_err_[kCallCount] = {};
  std::vector<int> filter_ids_;
  std::vector<std::string> filter_bdfs_;  // normalize_bdf form
  bool keep(int hip_id, const std::string& bdf) const {
    if (!has_device_filter()) return true;
    for (int x : filter_ids_)
      if (x == hip_id) return true;
    if (!bdf.empty()) {
      std::string b = normalize_bdf(bdf);
      for (const auto& x : filter_bdfs_)
        if (x == b) return true;
    }
    return false;
  }
};

// ---------------------------------------------------------------------------------------------
// Mock backend
// ---------------------------------------------------------------------------------------------
struct MockProc {
  uint32_t pid = 0;
  int device = 0;
  std::string name = "python3";
  double vram_bytes = 1024.0 * 1024 * 1024;
  double gfx_share = 0.5;  // fraction of device busy time attributed to this process
  bool kfd_only = false;   // HIP compute on KFD user queues: no DRM fdinfo engine time
  int queues = -1;         // hardware queues it holds on the device (ProcSample::queues; -1 unknown)
};

struct MockConfig {
  int gpus = 1;
  uint64_t seed = 1;
  std::string mode = "wave";          // "wave" (sinusoid), "const", "idle", "load"
  double const_util = 50.0;
  double hang_ms = 0.0;               // sleep inside sample() (watchdog / latency tests)
  int hang_device = -1;               // ... on this hip_id only (-1: every device)
  int fail_device = -1;               // device whose sample() fails ...
  int fail_every = 0;                 // ... every N calls (0 = never); -1 = always
  int procs_fail_every = 0;           // every device's processes() fails every N calls (0 = never)
  std::vector<std::string> unsupported;  // field names forced to NaN, e.g. "temp_edge"
  std::vector<MockProc> procs;
  int n_xcd = 8;
  int n_links = 7;
  double firmware_hz = 50.0;          // how fast the fake firmware table advances
  bool occupancy = true;              // KFD cu_occupancy readable (false: a node without the file)
  std::string link_order = "index";   // link-metrics entry order: index | reverse | rotate
  bool link_offset = false;           // entry counters with another origin than the table's (delta pairing only)
  bool full = false;                  // every scalar field filled (fan, voltages, ... that MI355X leaves N/A):
                                      // the metric reference lists the families a full table produces
};

class MockBackend : public Backend {
 public:
  explicit MockBackend(MockConfig cfg);
  std::string name() const override { return "mock"; }
  bool init(std::string* err) override;
  int device_count() const override { return static_cast<int>(devs_.size()); }
  const DeviceStatic& static_info(int i) const override { return devs_[i]; }
  void sample(int i, DeviceSample* out) override;
  bool processes(int i, std::vector<ProcSample>* out) override;
  bool supports_links() const override { return true; }
  void sample_links(int i, DeviceSample* out) override;
  bool supports_ras() const override { return true; }
  void sample_ras(int i, DeviceSample* out, int slice = 0, int nslices = 1) override;
  bool supports_occupancy(int) const override { return cfg_.occupancy; }
  bool concurrent_processes(int) const override { return true; }  // every call holds mu_
  void occupancy(int i, const std::vector<uint32_t>& pids, std::vector<double>* out) override;
  bool occupancy_scan(int i, std::vector<OccRead>* out) override;

  // Test controls (thread-safe).
  // Every cu_occupancy read of `dev` (process list and sub-samples alike) returns the next value of
  // `values`, cycling; empty = back to the util-proportional default.
  void set_occ_series(int dev, const std::vector<double>& values);
  uint64_t occ_reads(int dev) const;
  // Add errors to a RAS block of `dev` (blocks: umc gfx sdma mmhub xgmi_wafl vcn jpeg); `event`
  // counters: "fatal", "poison_created", "poison_consumed", "bad_pages" (set, not added).
  void add_ecc(int dev, const std::string& block, uint64_t ue, uint64_t ce, uint64_t de);
  void set_ras_event(int dev, const std::string& event, double value);
  void set_util(int dev, double pct);
  void set_procs(const std::vector<MockProc>& procs);
  void set_fail(int dev, int every);
  void set_hang_ms(double ms, int dev = -1);  // dev -1: every device
  // Force link `link` of `dev` to carry `gbps` GB/s of reads (and half of it as writes);
  // negative = back to the util-proportional default. For xGMI link-map tests.
  void set_xgmi(int dev, int link, double gbps);
  void set_link_up(int dev, int link, bool up);  // firmware link status (0 down) of one xGMI slot
  uint64_t link_calls(int dev) const;            // sample_links() calls (link-metrics refreshes)
  void set_link_fail(int dev, bool fail);        // link-metrics reads of `dev` fail (links_read -1)
  // The fake SMU of `dev` stops refreshing its table (firmware timestamp and accumulators hold) / resumes.
  void set_firmware_frozen(int dev, bool frozen);
  // The next `n` occupancy_scan() calls of `dev` fail as a transient error would (occupancy stays supported).
  void fail_scans(int dev, int n);
  // The next `n` processes() calls of `dev` fail as a transient library error would.
  void fail_procs(int dev, int n);
  uint64_t calls(int dev) const;
  bool prewarm(int i) override;
  uint64_t prewarms(int dev) const;  // prewarm() calls

 private:
  MockConfig cfg_;
  std::vector<DeviceStatic> devs_;
  mutable std::mutex mu_;
  std::vector<double> forced_util_;
  std::vector<std::vector<double>> occ_series_;  // per dev (set_occ_series)
  std::vector<uint64_t> occ_reads_;               // per dev: cu_occupancy reads served
  double occ_value(int i, const MockProc& p, double util);  // mu_ held
  std::vector<double> forced_xgmi_;  // per dev * kMaxLinks, GB/s (NaN = default)
  std::vector<char> link_down_;      // per dev * kMaxLinks
  std::vector<uint64_t> link_calls_;
  std::vector<char> link_fail_;
  std::vector<int64_t> frozen_tick_;
  std::vector<int> procs_fail_;      // per dev: process lists still to fail
  std::vector<uint64_t> procs_calls_;  // per dev: processes() calls (procs_fail_every)
  std::vector<int> scan_fail_;       // per dev: occupancy scans still to fail  // per dev: firmware tick the fake SMU is stuck at (-1 = running)
  std::vector<uint64_t> calls_, prewarms_;
  std::vector<uint64_t> energy_, xgmi_rd_, xgmi_wr_, busy_acc_, acc_counter_, gfx_act_acc_, pcie_acc_;
  std::vector<uint64_t> lim_acc_;  // per device x XCC x {ppt, thermal, any, low-util}
  std::vector<RasSample> ras_;     // per device (mock RAS state)
  std::map<std::pair<uint32_t, int>, uint64_t> proc_gfx_ns_;
  int64_t t0_ns_ = 0;
  std::vector<int64_t> last_ns_;
};

// ---------------------------------------------------------------------------------------------
// amdsmi backend (dlopen'd libamd_smi)
// ---------------------------------------------------------------------------------------------
struct SmiTable;  // smi_table.h
class SysfsGpu;   // sysfs_fast.h

class AmdSmiBackend : public Backend {
 public:
  explicit AmdSmiBackend(std::string lib_path = "");
  ~AmdSmiBackend() override;
  std::string name() const override { return "amdsmi"; }
  bool init(std::string* err) override;
  void shutdown() override;
  int device_count() const override { return static_cast<int>(devs_.size()); }
  const DeviceStatic& static_info(int i) const override { return devs_[i]; }
  void sample(int i, DeviceSample* out) override;
  bool processes(int i, std::vector<ProcSample>* out) override;
  bool supports_processes(int i) const override;
  bool supports_links() const override;
  void sample_links(int i, DeviceSample* out) override;
  bool supports_ras() const override { return true; }
  void sample_ras(int i, DeviceSample* out, int slice = 0, int nslices = 1) override;
  bool supports_occupancy(int i) const override;  // with the sysfs fast path (KFD files)
  // sysfs fast path: the table pread and the KFD / fdinfo reads share no state
  bool concurrent_processes(int i) const override { return supports_occupancy(i); }
  void set_tick_occupancy(bool on) override { tick_occupancy_ = on; }
  void maintain(int i) override;                   // fast path: due /proc fd-table refreshes
  bool prewarm(int i) override;                    // fast path: one throwaway gpu_metrics pread
  void occupancy(int i, const std::vector<uint32_t>& pids, std::vector<double>* out) override;
  bool occupancy_scan(int i, std::vector<OccRead>* out) override;
  std::string lib_version() const { return lib_version_; }
  // Expose every physical device `r` times (distinct gpu_id labels). Only for measuring how the
  // sampler scales with the GPU count on a box with fewer GPUs than a full 8x MI355X node.
  void set_replicate(int r) { replicate_ = r < 1 ? 1 : r; }
  // Direct sysfs/KFD reads for the per-tick values (sysfs_fast.h); libamd_smi stays the source of
  // enumeration, statics, links and the fallback. Applied at init().
  void set_fast_path(bool on, std::string sys_root = "/sys", std::string proc_root = "/proc") {
    fast_path_ = on;
    sys_root_ = std::move(sys_root);
    proc_root_ = std::move(proc_root);
  }
  int fast_path_devices() const;
  // KFD per-pid files kept open across the fast-path GPUs, and reads served from them
  void kfd_file_stats(uint64_t* open_fds, uint64_t* cached_reads) const;
  const std::string& fast_path_status() const { return fast_status_; }
  // Field-by-field libamd_smi vs sysfs-decoded firmware table of device i: (field, amdsmi, sysfs).
  std::vector<std::tuple<std::string, double, double>> compare_tables(int i, std::string* err);

 private:
  bool validate_fast(int i, std::string* why);
  int replicate_ = 1;
  bool fast_path_ = true;
  std::atomic<bool> tick_occupancy_{true};
  std::string sys_root_ = "/sys", proc_root_ = "/proc", fast_status_;
  std::vector<std::unique_ptr<SysfsGpu>> fast_;
  std::vector<uint64_t> kfd_ids_;
  std::string lib_path_;
  std::unique_ptr<SmiTable> t_;
  bool inited_ = false;
  std::vector<void*> handles_;
  std::vector<DeviceStatic> devs_;
  std::string lib_version_;
  double energy_res_uj_ = 15.3;  // amdsmi_get_energy_count counter_resolution (MI355X: 15.3 uJ)
  // Per device: calls that returned NOT_SUPPORTED are not retried.
  struct Caps {
    bool metrics = true, vram = true, activity = true, power = true, procs = true, links = true;
    bool ras_sysfs = true;          // ras/ directory present (else amdsmi ECC calls)
    uint64_t ecc_blocks = ~0ull;    // AMDSMI_GPU_BLOCK_* bits still worth asking for
    uint64_t ecc_seen = 0;          // ... and those that answered at least once
  };
  std::vector<Caps> caps_;
  std::vector<std::unique_ptr<RasSysfsReader>> ras_readers_;  // per device, created on first use
  std::vector<RasRetry> ras_retry_;                           // per device: transient-failure backoff
  std::vector<std::vector<char>> proc_buf_;  // reusable process-list buffers
};

// ---------------------------------------------------------------------------------------------
// rocm_smi_lib fallback (dlopen'd librocm_smi64), same firmware table
// ---------------------------------------------------------------------------------------------
struct RsmiTable;

class RocmSmiBackend : public Backend {
 public:
  explicit RocmSmiBackend(std::string lib_path = "");
  ~RocmSmiBackend() override;
  std::string name() const override { return "rocm_smi"; }
  bool init(std::string* err) override;
  void shutdown() override;
  int device_count() const override { return static_cast<int>(devs_.size()); }
  const DeviceStatic& static_info(int i) const override { return devs_[i]; }
  void sample(int i, DeviceSample* out) override;
  bool processes(int i, std::vector<ProcSample>* out) override;
  bool supports_processes(int i) const override;  // the library exports the compute-process calls
  bool supports_ras() const override { return true; }
  void sample_ras(int i, DeviceSample* out, int slice = 0, int nslices = 1) override;  // kernel ras/ sysfs files
  std::string lib_version() const { return lib_version_; }
  void set_sys_root(std::string r) { sys_root_ = std::move(r); }

 private:
  std::string sys_root_ = "/sys";
  std::string lib_path_;
  std::unique_ptr<RsmiTable> t_;
  bool inited_ = false;
  bool metrics_ok_ = true;
  std::vector<DeviceStatic> devs_;
  std::vector<uint32_t> idx_;  // rsmi device index per exported device
  std::vector<std::unique_ptr<RasSysfsReader>> ras_readers_;
  std::vector<char> ras_missing_;  // per device: no ras/ error-count files (reset by init())
  std::vector<RasRetry> ras_retry_;  // per device: backoff after transient read failures
  std::string lib_version_;
  double energy_res_uj_ = 15.3;
};

std::unique_ptr<Backend> make_backend(const std::string& spec, std::string* err);

// Field-name registry (used by mock "unsupported" lists and tests).
int field_by_name(const std::string& name);
const char* field_name(int f);

}  // namespace gpumon
