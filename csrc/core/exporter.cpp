#include "exporter.h"
#include "tls.h"

#include <pthread.h>
#include <sched.h>
#include <sys/prctl.h>

#include <dirent.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <functional>
#include <unordered_set>

#include "common.h"
#include "docker_lite.h"
#include "grpc_lite.h"
#include "http_client.h"
#include "kubelet_files.h"
#include "ondevice.h"
#include "trace.h"
#include "xgmi_map.h"

namespace gpumon {

// ---------------------------------------------------------------------------------------------
// Per-device sampling workers with a watchdog.
//
// Each GPU gets its own thread; a tick hands every idle worker a request and waits until all
// answer or `device_timeout_s` passes. A device whose call has not returned by then (a hung
// driver/SMU call) is exported as gpu_up 0 with gpumon_device_timeouts_total incremented, and is not
// asked again until its call returns -- the other GPUs keep their 1 Hz cadence (the reference
// stalled the whole node on any slow nvidia-smi, gpu.py:104-116). Workers only touch their own
// heap state and the backend, so a worker stuck at shutdown can be detached safely (the backend is
// then deliberately leaked instead of destroyed under it).
// ---------------------------------------------------------------------------------------------
struct Exporter::DoneSignal {
  std::mutex mu;
  std::condition_variable cv;
};

struct Exporter::DevWorker {
  std::mutex mu;
  std::condition_variable cv;
  bool quit = false;
  bool pending = false;          // request posted, not yet picked up
  bool busy = false;             // request in flight (posted or running)
  uint64_t req = 0;              // tick id of the current request
  std::atomic<uint64_t> done{0}; // tick id whose results are stored below
  bool want_links = false, want_procs = false, want_ras = false;
  bool ras_async = false;        // read the RAS slice AFTER publishing this tick (applied next tick)
  int ras_slice = 0, ras_n = 1;
  int64_t started_ns = 0;
  int64_t picked_ns = 0, device_ns = 0;  // pickup time and device-call time of the stored tick
  DeviceSample sample;
  std::vector<ProcSample> procs;
  int64_t proc_ns = 0;
  std::thread th;
};

// Between ticks the worker sub-samples the KFD cu_occupancy of the processes its device had at
// the last tick, every occ_period_ns (interval / occ_samples): one read per tick is an instant
// (4.6 % of reads under a saturating burn land between two kernels and return 0, profiles/
// r2_kfd_occupancy.md); the tick's process rows carry the interval mean and the share of reads
// that found the process's waves resident.
// SCHED_FIFO for the calling thread (rt_priority); counted in `rt` while the thread lives.
static bool apply_rt(int prio, const std::string& who, std::atomic<int>* rt) {
  if (prio <= 0) return false;
  sched_param sp{};
  sp.sched_priority = std::clamp(prio, 1, 99);
  const int rc = pthread_setschedparam(pthread_self(), SCHED_FIFO, &sp);
  if (rc != 0) {
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true))
      GPUMON_LOG(LogLevel::kWarn, "exporter",
                 "rt_priority " + std::to_string(prio) + " for " + who + ": " + strerror(rc) +
                     " (needs CAP_SYS_NICE); sampling threads keep normal scheduling");
    return false;
  }
  rt->fetch_add(1);
  return true;
}

static void read_process_stats(SelfStats* s);  // /proc/self figures (defined below)

static void dev_worker_main(std::shared_ptr<Exporter::DevWorker> w, std::shared_ptr<Exporter::DoneSignal> sig,
                            Backend* backend, int i, int64_t occ_period_ns,
                            std::shared_ptr<std::atomic<uint64_t>> occ_reads,
                            std::shared_ptr<std::atomic<uint64_t>> scan_failures, int rt_prio,
                            std::shared_ptr<std::atomic<int>> rt_threads,
                            std::shared_ptr<std::atomic<int64_t>> next_tick, int64_t prewarm_ns) {
  set_thread_name("gpumon-dev" + std::to_string(i));
  const bool rt = apply_rt(rt_prio, "device worker", rt_threads.get());
  struct RtCount {  // the gauge counts live threads
    bool on;
    std::atomic<int>* n;
    ~RtCount() {
      if (on) n->fetch_sub(1);
    }
  } rt_count{rt, rt_threads.get()};
  std::vector<uint32_t> occ_pids;                      // processes on this device at the last tick
  std::vector<double> occ_sum;                         // per occ_pids entry
  std::vector<int> occ_n, occ_busy;
  std::vector<double> vals;
  std::vector<OccRead> scan;
  const bool occ_on = occ_period_ns > 0 && backend->supports_occupancy(i);
  // The sub-samples list the device's processes themselves where the backend can (KFD proc dir):
  // a tenant that started since the last tick is read from then on, not from the next tick (a
  // 10 %-resident arrival otherwise had one read in its first interval).
  bool scan_ok = occ_on;
  // A failed listing (a transient opendir / read error) is retried with a backoff (1 s doubling to
  // 60 s), not latched off for the worker's life; only a backend that stopped supporting the read
  // ends the scans. In between, the known pids are re-read as before.
  int64_t scan_retry_at = 0, scan_backoff_ns = 1'000'000'000;
  // Every 4th sub-sample lists the directory (new tenants show up within 4 periods, 0.2 s at 1 Hz);
  // the others re-read the known pids only: a node-wide KFD listing per GPU per sub-sample would
  // cost P opens each time on a node with P GPU processes.
  constexpr int kScanEvery = 4;
  uint64_t n_sub = 0;
  int64_t next_occ = 0;
  // Prewarm: one throwaway firmware-table read prewarm_ns before each tick's deadline, so the
  // tick's own read finds the SMU's fetch path awake (~50 us instead of 150-300 us after a long
  // gap, profiles/r3_capacity.md). Once per deadline; skipped when the deadline is already close.
  int64_t warmed_for = 0;
  // The process list (KFD + fdinfo reads, ~0.1 ms) runs on a second thread while this one reads
  // the firmware table (~0.2 ms, mostly the SMU fetch): the device's part of a tick becomes the
  // longer of the two instead of their sum. Only where the backend allows it (sysfs fast path).
  struct ProcJob {
    std::mutex mu;
    std::condition_variable cv;
    bool want = false, done = false, quit = false;
    std::vector<ProcSample> out;
    bool ok = false;
    int64_t ns = 0;
  };
  std::shared_ptr<ProcJob> job;
  std::thread proc_thread;
  if (backend->concurrent_processes(i)) {
    job = std::make_shared<ProcJob>();
    proc_thread = std::thread([job, backend, i] {
      set_thread_name("gpumon-proc" + std::to_string(i));
      std::unique_lock<std::mutex> lk(job->mu);
      for (;;) {
        job->cv.wait(lk, [&] { return job->want || job->quit; });
        if (job->quit) return;
        job->want = false;
        lk.unlock();
        std::vector<ProcSample> p;
        const int64_t t = mono_ns();
        const bool ok = backend->processes(i, &p);
        const int64_t ns = mono_ns() - t;
        lk.lock();
        job->out = std::move(p);
        job->ok = ok;
        job->ns = ns;
        job->done = true;
        job->cv.notify_all();
      }
    });
  }
  struct ProcJoin {  // every return path: stop and join the process-list thread
    std::shared_ptr<ProcJob>& job;
    std::thread& th;
    ~ProcJoin() {
      if (!job) return;
      {
        std::lock_guard<std::mutex> g(job->mu);
        job->quit = true;
      }
      job->cv.notify_all();
      if (th.joinable()) th.join();
    }
  } proc_join{job, proc_thread};
  // RAS refreshes read off the tick's critical path: the worker reads the slice right after it
  // published the tick (the files cost 0.25-0.5 ms under load: the slowest tick of every RAS pass,
  // profiles/r2_bench.md) and the next tick carries the result.
  RasSample ras_ready;
  bool have_ras_ready = false;
  uint64_t jitter = 0x9E3779B97F4A7C15ull * static_cast<uint64_t>(i + 1);  // per-worker LCG state
  while (true) {
    uint64_t id;
    bool links, procs, ras, ras_async;
    int ras_slice, ras_n;
    {
      std::unique_lock<std::mutex> lk(w->mu);
      bool subsample = false, warm = false;
      while (!w->quit && !w->pending) {
        const int64_t now = mono_ns();
        int64_t wake = INT64_MAX;
        if (prewarm_ns > 0) {
          const int64_t nt = next_tick->load(std::memory_order_acquire);
          if (nt > 0 && nt != warmed_for) {
            if (now >= nt - prewarm_ns) {
              warmed_for = nt;
              if (now < nt - prewarm_ns / 4) {  // not when the tick is about to sample anyway
                warm = true;
                break;
              }
            } else {
              wake = nt - prewarm_ns;
            }
          }
        }
        if (occ_on && !(occ_pids.empty() && !scan_ok)) {
          if (next_occ <= now) {
            subsample = true;
            break;
          }
          wake = std::min(wake, next_occ);
        }
        if (wake == INT64_MAX) {
          w->cv.wait(lk);
          continue;
        }
        // system_clock slices checked against the monotonic deadline (TSan: see sample_devices)
        w->cv.wait_until(lk, std::chrono::system_clock::now() +
                                 std::chrono::nanoseconds(std::min<int64_t>(wake - now, 20'000'000)));
      }
      if (w->quit) return;
      if (warm) {
        lk.unlock();
        TraceRange tr("gpumon.prewarm");
        backend->prewarm(i);
        continue;
      }
      if (subsample) {
        lk.unlock();
        const bool scan_turn = scan_ok && (n_sub++ % kScanEvery == 0) && mono_ns() >= scan_retry_at;
        bool scanned = false;
        if (scan_turn) {
          scanned = backend->occupancy_scan(i, &scan);
          scan_failures->fetch_add(scanned ? 0 : 1, std::memory_order_relaxed);
          if (scanned) {
            scan_backoff_ns = 1'000'000'000;
          } else if (!backend->supports_occupancy(i)) {
            scan_ok = false;
          } else {
            scan_retry_at = mono_ns() + scan_backoff_ns;
            scan_backoff_ns = std::min<int64_t>(scan_backoff_ns * 2, 60'000'000'000);
          }
        }
        if (scanned) {
          vals.assign(occ_pids.size(), kNaN);
          for (const OccRead& r : scan) {
            size_t k = std::find(occ_pids.begin(), occ_pids.end(), r.pid) - occ_pids.begin();
            if (k == occ_pids.size()) {  // arrived since the last tick
              occ_pids.push_back(r.pid);
              occ_sum.push_back(0.0);
              occ_n.push_back(0);
              occ_busy.push_back(0);
              vals.push_back(kNaN);
            }
            vals[k] = r.cu_occupancy;
          }
          occ_reads->fetch_add(scan.size(), std::memory_order_relaxed);
        } else {
          backend->occupancy(i, occ_pids, &vals);
          occ_reads->fetch_add(occ_pids.size(), std::memory_order_relaxed);
        }
        for (size_t k = 0; k < occ_pids.size() && k < vals.size(); ++k)
          if (has(vals[k])) {
            occ_sum[k] += vals[k];
            occ_n[k]++;
            occ_busy[k] += vals[k] > 0 ? 1 : 0;
          }
        // jittered spacing (0.5-1.5 periods, same mean): fixed-period reads phase-lock to a
        // periodic workload (host-synchronised batches) and keep hitting -- or missing -- its gaps
        jitter = jitter * 6364136223846793005ull + 1442695040888963407ull;
        const double u = static_cast<double>(jitter >> 11) * (1.0 / 9007199254740992.0);
        next_occ += static_cast<int64_t>(occ_period_ns * (0.5 + u));
        if (next_occ < mono_ns()) next_occ = mono_ns() + occ_period_ns;
        continue;
      }
      w->pending = false;
      w->picked_ns = mono_ns();
      id = w->req;
      links = w->want_links;
      procs = w->want_procs;
      ras = w->want_ras;
      ras_async = w->ras_async;
      ras_slice = w->ras_slice;
      ras_n = w->ras_n;
    }
    DeviceSample s;
    std::vector<ProcSample> p;
    int64_t pns = 0;
    const int64_t t_dev0 = mono_ns();
    {
      TraceRange tr("gpumon.sample_dev");
      const bool overlap = procs && job;
      if (overlap) {
        std::lock_guard<std::mutex> g(job->mu);
        job->want = true;
        job->done = false;
      }
      if (overlap) job->cv.notify_all();
      backend->sample(i, &s);
      if (links) backend->sample_links(i, &s);
      if (have_ras_ready && s.ok) {
        s.ras = std::move(ras_ready);
        have_ras_ready = false;
      }
      if (ras && !ras_async && s.ok) backend->sample_ras(i, &s, ras_slice, ras_n);
      if (overlap) {
        std::unique_lock<std::mutex> lk(job->mu);
        job->cv.wait(lk, [&] { return job->done; });
        if (s.ok) {
          p = std::move(job->out);
          pns = job->ns;
          s.procs_read = job->ok ? 1 : backend->supports_processes(i) ? -1 : 0;
        }
        job->out.clear();
      } else if (procs && s.ok) {
        const int64_t t = mono_ns();
        const bool ok = backend->processes(i, &p);
        pns = mono_ns() - t;
        s.procs_read = ok ? 1 : backend->supports_processes(i) ? -1 : 0;
      }
    }
    const bool ok_for_ras = s.ok;
    const int64_t dev_ns = mono_ns() - t_dev0;
    // fold the interval's sub-samples into this tick's reading (with sub-sampling on, the tick's
    // process list skips its own cu_occupancy read: Exporter::start_workers, set_tick_occupancy)
    for (auto& ps : p) {
      if (!has(ps.cu_occupancy) && !occ_on) continue;
      double sum = has(ps.cu_occupancy) ? ps.cu_occupancy : 0.0;
      int n = has(ps.cu_occupancy) ? 1 : 0, busy = ps.cu_occupancy > 0 ? 1 : 0;
      for (size_t k = 0; k < occ_pids.size(); ++k)
        if (occ_pids[k] == ps.pid) {
          sum += occ_sum[k];
          n += occ_n[k];
          busy += occ_busy[k];
          break;
        }
      ps.cu_occupancy = n > 0 ? sum / n : kNaN;
      ps.occ_samples = n;
      ps.occ_busy = busy;
    }
    // A listed process that arrived since the last list (no sub-sample could know it) gets one read
    // now, so its first row is not empty. Only new pids: a known pid whose reads keep returning
    // nothing (NaN) would otherwise cost an extra open on the tick's path every tick.
    if (occ_on) {
      std::vector<uint32_t> unread;
      for (const auto& ps : p)
        if (ps.occ_samples == 0 && std::find(occ_pids.begin(), occ_pids.end(), ps.pid) == occ_pids.end())
          unread.push_back(ps.pid);
      if (!unread.empty()) {
        backend->occupancy(i, unread, &vals);
        occ_reads->fetch_add(unread.size(), std::memory_order_relaxed);
        size_t k = 0;
        for (auto& ps : p)
          if (ps.occ_samples == 0 && k < vals.size() && ps.pid == unread[k]) {
            const double v = vals[k++];
            if (!has(v)) continue;
            ps.cu_occupancy = v;
            ps.occ_samples = 1;
            ps.occ_busy = v > 0 ? 1 : 0;
          }
      }
    }
    // a failed tick (or a failed process list) listed nothing: keep sub-sampling the known pids.
    // The sums restart every tick either way: a failed list's interval is not folded into the next
    // good tick's mean (two intervals averaged as one); the held rows carry no occupancy.
    if (occ_on && procs && ok_for_ras && s.procs_read >= 0) {
      occ_pids.clear();
      for (const auto& ps : p)
        if (std::find(occ_pids.begin(), occ_pids.end(), ps.pid) == occ_pids.end()) occ_pids.push_back(ps.pid);
      next_occ = mono_ns() + occ_period_ns;
    }
    if (occ_on && procs) {
      occ_sum.assign(occ_pids.size(), 0.0);
      occ_n.assign(occ_pids.size(), 0);
      occ_busy.assign(occ_pids.size(), 0);
    }
    {
      std::lock_guard<std::mutex> g(w->mu);
      w->sample = std::move(s);
      w->procs = std::move(p);
      w->proc_ns = pns;
      w->device_ns = dev_ns;
      w->busy = false;
      w->done.store(id, std::memory_order_release);
      if (w->quit) {
        std::lock_guard<std::mutex> g2(sig->mu);
        sig->cv.notify_all();
        return;
      }
    }
    {
      std::lock_guard<std::mutex> g(sig->mu);
      sig->cv.notify_all();
    }
    if (ras && ras_async && ok_for_ras) {
      TraceRange tr("gpumon.ras_async");
      DeviceSample scratch;
      backend->sample_ras(i, &scratch, ras_slice, ras_n);
      if (scratch.ras.valid) {
        ras_ready = std::move(scratch.ras);
        have_ras_ready = true;
      }
    }
    if (procs) backend->maintain(i);
  }
}

void Exporter::start_workers(int n) {
  stop_workers();
  if (!done_sig_) done_sig_ = std::make_shared<DoneSignal>();
  for (int i = 0; i < n; ++i) {
    auto w = std::make_shared<DevWorker>();
    // sub-sample period: interval / occ_samples, no faster than 50 Hz; manual ticks: none
    const int64_t occ_ns = cfg_.interval_s > 0 && cfg_.occ_samples > 1 && cfg_.processes
                               ? std::max<int64_t>(20'000'000, static_cast<int64_t>(cfg_.interval_s * 1e9 / cfg_.occ_samples))
                               : 0;
    // the workers' sub-samples stand in for the tick's own cu_occupancy read (the costliest
    // per-process file: ~27 us, a KFD walk over the process's queues)
    if (i == 0) backend_->set_tick_occupancy(occ_ns == 0 || !backend_->supports_occupancy(i));
    // prewarm only at intervals >= 20 ms: a read within ~5 ms of the last one is warm already, and
    // the lead is capped at a quarter of the interval
    const int64_t prewarm_ns = cfg_.interval_s >= 0.02 && cfg_.prewarm_ms > 0
                                   ? static_cast<int64_t>(std::min(cfg_.prewarm_ms, cfg_.interval_s * 250.0) * 1e6)
                                   : 0;
    w->th = std::thread(dev_worker_main, w, done_sig_, backend_.get(), i, occ_ns, occ_reads_, scan_failures_,
                        cfg_.rt_priority,
                        rt_threads_, next_tick_ns_, prewarm_ns);
    workers_.push_back(std::move(w));
  }
}

// Returns false if a worker was stuck in a device call and had to be detached.
bool Exporter::stop_workers() {
  bool clean = true;
  for (auto& w : workers_) {
    bool busy;
    {
      std::lock_guard<std::mutex> g(w->mu);
      w->quit = true;
      busy = w->busy && !w->pending;
    }
    w->cv.notify_all();
    if (busy) {
      // give an in-flight call a moment to return before giving up on it
      const int64_t until = mono_ns() + 200'000'000;
      while (mono_ns() < until) {
        {
          std::lock_guard<std::mutex> g(w->mu);
          if (!w->busy) break;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
      std::lock_guard<std::mutex> g(w->mu);
      busy = w->busy;
    }
    if (busy) {
      GPUMON_LOG(LogLevel::kError, "exporter", "device worker stuck in a backend call at shutdown: detaching it");
      w->th.detach();
      clean = false;
    } else if (w->th.joinable()) {
      w->th.join();
    }
  }
  workers_.clear();
  return clean;
}

bool Exporter::workers_busy() const {
  for (const auto& w : workers_) {
    std::lock_guard<std::mutex> g(w->mu);
    if (w->busy) return true;
  }
  return false;
}

// ---------------------------------------------------------------------------------------------
static MockConfig parse_mock_spec(const std::string& spec, MockConfig base) {
  // "mock" or "mock:gpus=8,mode=load,n_xcd=8,fail_device=1,fail_every=3,hang_ms=5,unsupported=a;b,procs=2"
  size_t colon = spec.find(':');
  if (colon == std::string::npos) return base;
  int procs_per_gpu = 0;
  for (const auto& kv : split(spec.substr(colon + 1), ',')) {
    size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
    if (k == "gpus") base.gpus = atoi(v.c_str());
    else if (k == "mode") base.mode = v;
    else if (k == "const_util") base.const_util = atof(v.c_str());
    else if (k == "n_xcd") base.n_xcd = atoi(v.c_str());
    else if (k == "n_links") base.n_links = atoi(v.c_str());
    else if (k == "fail_device") base.fail_device = atoi(v.c_str());
    else if (k == "fail_every") base.fail_every = atoi(v.c_str());
    else if (k == "procs_fail_every") base.procs_fail_every = std::max(0, atoi(v.c_str()));
    else if (k == "hang_ms") base.hang_ms = atof(v.c_str());
    else if (k == "hang_device") base.hang_device = atoi(v.c_str());
    else if (k == "seed") base.seed = strtoull(v.c_str(), nullptr, 10);
    else if (k == "firmware_hz") base.firmware_hz = atof(v.c_str());
    else if (k == "occupancy") base.occupancy = atoi(v.c_str()) != 0;
    else if (k == "link_order") base.link_order = v;
    else if (k == "link_offset") base.link_offset = atoi(v.c_str()) != 0;
    else if (k == "full") base.full = atoi(v.c_str()) != 0;
    else if (k == "unsupported") base.unsupported = split(v, ';');
    else if (k == "procs") procs_per_gpu = std::max(0, atoi(v.c_str()));
  }
  // procs=N: N processes on every GPU (the exporter's own pid first, so one attributes; the rest
  // are pids that do not exist), half of them KFD-only -- sharing, occupancy sub-samples and the
  // process-list thread from the command line (sanitizer runs)
  for (int d = 0; d < base.gpus; ++d)
    for (int k = 0; k < procs_per_gpu; ++k) {
      MockProc p;
      p.pid = k == 0 ? static_cast<uint32_t>(getpid()) : static_cast<uint32_t>(3900000 + d * 100 + k);
      p.device = d;
      p.name = "mock-tenant-" + std::to_string(k);
      p.vram_bytes = static_cast<double>(1 + k) * (1ull << 30);
      p.gfx_share = 1.0 / procs_per_gpu;
      p.kfd_only = k % 2 == 1;
      base.procs.push_back(p);
    }
  return base;
}

std::unique_ptr<Backend> make_backend_from_config(const ExporterConfig& cfg, std::string* err) {
  std::unique_ptr<Backend> b;
  if (starts_with(cfg.backend, "mock")) {
    b = std::make_unique<MockBackend>(parse_mock_spec(cfg.backend, cfg.mock));
  } else if (starts_with(cfg.backend, "amdsmi") || cfg.backend == "auto") {
    auto a = std::make_unique<AmdSmiBackend>(cfg.amdsmi_lib);
    // "amdsmi:replicate=8": sample every real device 8 times (scaling rehearsal on small boxes)
    size_t p = cfg.backend.find("replicate=");
    if (p != std::string::npos) a->set_replicate(atoi(cfg.backend.c_str() + p + 10));
    a->set_fast_path(cfg.fast_path, cfg.sysfs_root, cfg.attribution.procfs_root);
    b = std::move(a);
  } else if (cfg.backend == "rocm_smi") {
    auto r = std::make_unique<RocmSmiBackend>(cfg.rocm_smi_lib);
    r->set_sys_root(cfg.sysfs_root);
    b = std::move(r);
  } else {
    if (err) *err = "unknown backend '" + cfg.backend + "' (amdsmi | rocm_smi | mock[:k=v,...] | auto)";
    return nullptr;
  }
  b->set_device_filter(cfg.devices);
  return b;
}

std::unique_ptr<Backend> make_backend(const std::string& spec, std::string* err) {
  ExporterConfig c;
  c.backend = spec;
  return make_backend_from_config(c, err);
}

// ---------------------------------------------------------------------------------------------
Exporter::Exporter(ExporterConfig cfg)
    : cfg_(std::move(cfg)), sample_hist_(latency_buckets()), scrape_hist_(latency_buckets()) {
  if (cfg_.host.empty()) cfg_.host = "no_name";
  // Mock processes are fake PIDs: there is no /dev/kfd handle to verify.
  if (starts_with(cfg_.backend, "mock")) cfg_.attribution.verify_kfd = false;
  attr_ = std::make_unique<Attributor>(cfg_.attribution);
}

Exporter::~Exporter() { stop(); }

bool Exporter::ensure_backend() {
  if (backend_up_) return true;
  int64_t now = mono_ns();
  if (now < next_init_ns_) return false;
  next_init_ns_ = now + static_cast<int64_t>(cfg_.init_retry_s * 1e9);
  std::string err;
  if (!backend_) backend_ = make_backend_from_config(cfg_, &err);
  bool ok = backend_ && backend_->init(&err);
  if (!ok && cfg_.backend == "auto" && backend_ && backend_->name() == "amdsmi") {
    // auto: libamd_smi missing or failing -> rocm_smi_lib behind the same kind of dlopen table
    auto fb = std::make_unique<RocmSmiBackend>(cfg_.rocm_smi_lib);
    fb->set_device_filter(cfg_.devices);
    fb->set_sys_root(cfg_.sysfs_root);
    std::string err2;
    if (fb->init(&err2)) {
      GPUMON_LOG(LogLevel::kWarn, "exporter", "amdsmi unavailable (" + err + "); using rocm_smi fallback");
      backend_ = std::move(fb);
      ok = true;
    } else {
      err += "; rocm_smi fallback: " + err2;
    }
  }
  if (!ok) {
    if (err != backend_error()) GPUMON_LOG(LogLevel::kError, "exporter", "backend init failed: " + err);
    std::lock_guard<std::mutex> g(err_mu_);
    backend_err_ = err;
    return false;
  }
  {
    std::lock_guard<std::mutex> g(err_mu_);
    backend_err_.clear();
  }
  std::vector<DeviceStatic> st;
  for (int i = 0; i < backend_->device_count(); ++i) st.push_back(backend_->static_info(i));
  {
    auto fresh = std::make_shared<TickState>();
    fresh->samples.assign(st.size(), DeviceSample{});
    fresh->rates.assign(st.size(), DeviceRates{});
    fresh->proc_counts.assign(st.size(), 0);
    fresh->procs.assign(st.size(), {});
    std::lock_guard<std::mutex> g(state_mu_);
    statics_ = std::make_shared<const std::vector<DeviceStatic>>(st);
    state_ = std::move(fresh);
    last_ok_.clear();  // a re-initialised backend may number its devices differently
    last_procs_.clear();
    xgmi_maps_.assign(st.size(), XgmiSlotMap{});
    dev_errors_.assign(st.size(), 0);
    dev_timeouts_.assign(st.size(), 0);
  }
  // One worker per GPU (parallel + watchdog) unless sequential sampling was asked for
  // (sample_threads 0) or the watchdog is disabled (device_timeout_s <= 0).
  if (cfg_.sample_threads != 0 && cfg_.device_timeout_s > 0) start_workers(static_cast<int>(st.size()));
  backend_up_ = true;
  GPUMON_LOG(LogLevel::kInfo, "exporter",
             "backend " + backend_->name() + " up with " + std::to_string(st.size()) + " GPU(s)");
  return true;
}

bool Exporter::start(std::string* err) {
  if (running_) return true;
  // An Influx push the exporter cannot perform is a configuration error, reported before anything
  // starts: the reference's requests.post took any http(s) URL (gpu.py:20,145), so an https:// or
  // mistyped INFLUXDB_URL must not leave a running exporter that silently never pushes.
  const std::string perr = check_push_config(cfg_.influx_url, cfg_.influx_token, influx_tls());
  if (!perr.empty()) {
    if (err) *err = perr;
    return false;
  }
  const char* rx = getenv("GPUMON_ROCTX");
  if (cfg_.roctx || (rx && *rx && strcmp(rx, "0") != 0)) {
    if (!Roctx::enable(true)) GPUMON_LOG(LogLevel::kWarn, "exporter", "roctx requested but librocprofiler-sdk-roctx not found");
  }
  if (!ensure_backend() && cfg_.backend != "auto" && !starts_with(cfg_.backend, "mock")) {
    // explicit amdsmi: keep running (retry with backoff) but report the error to the caller
    if (err) *err = backend_error();
  }
  if (!backend_up_ && starts_with(cfg_.backend, "mock")) {
    if (err) *err = backend_error();
    return false;
  }
  if (cfg_.serve_http) {
    server_ = std::make_unique<HttpServer>(
        cfg_.listen_addr, cfg_.port, cfg_.http_threads,
        [this](const HttpRequest& r, HttpResponse* w) { handle_http(r, w); },
        [this](const std::string& path, double s) {
          if (path == "/metrics") scrape_hist_.observe(s);
        });
    server_->set_rt(cfg_.http_rt_priority, cfg_.http_rt_budget);
    std::string e;
    if (!server_->start(&e)) {
      if (err) *err = e;
      server_.reset();
      return false;
    }
  }
  if (cfg_.interval_s > 0 && cfg_.interval_s < 0.02 && !starts_with(cfg_.backend, "mock"))
    GPUMON_LOG(LogLevel::kWarn, "exporter",
               "interval " + std::to_string(cfg_.interval_s * 1e3) +
                   " ms is below the firmware's gpu_metrics refresh (20 ms on MI355X): faster samples repeat the "
                   "last table (gpumon_stale_samples_total)");
  running_ = true;
  // First tick synchronously so /metrics is ready as soon as start() returns.
  tick();
  if (cfg_.interval_s > 0) sampler_ = std::thread([this] {
    set_thread_name("gpumon-sampler");
    sampler_loop();
  });
  if (!cfg_.influx_url.empty()) pusher_ = std::thread([this] {
    set_thread_name("gpumon-influx");
    influx_loop();
  });
  if (!cfg_.pod_resources_socket.empty() || !cfg_.cri_socket.empty() || !cfg_.docker_socket.empty() ||
      !cfg_.pod_log_root.empty() || !cfg_.device_checkpoint.empty()) {
    // metadata and allocations known before the first scrape
    if (!cfg_.cri_socket.empty()) cri_poll_once();
    if (!cfg_.docker_socket.empty()) docker_poll_once();
    if (!cfg_.pod_log_root.empty() || !cfg_.device_checkpoint.empty()) files_poll_once();
    if (!cfg_.pod_resources_socket.empty()) podres_poll_once();
    podres_ = std::thread([this] {
      set_thread_name("gpumon-k8s");
      podres_loop();
    });
  }
  return true;
}

void Exporter::stop() {
  // Also after a start() that failed part-way (e.g. the listen address): the backend and its
  // device workers were already up, and must not outlive the exporter.
  const bool was_running = running_.exchange(false);
  if (!was_running && !server_ && workers_.empty() && !backend_up_) return;
  seq_cv_.notify_all();
  push_cv_.notify_all();
  if (sampler_.joinable()) sampler_.join();
  if (pusher_.joinable()) pusher_.join();
  podres_cv_.notify_all();
  if (podres_.joinable()) podres_.join();
  if (server_) server_->stop();
  server_.reset();
  if (!stop_workers() && backend_) {
    // a detached worker is still inside a backend call: never destroy the backend under it
    (void)backend_.release();
  }
  if (backend_) backend_->shutdown();
  backend_up_ = false;
}

std::vector<TickInfo> Exporter::tick_log() const {
  std::lock_guard<std::mutex> g(tick_log_mu_);
  if (tick_log_.size() < kTickLog) return tick_log_;
  std::vector<TickInfo> v(tick_log_.begin() + static_cast<std::ptrdiff_t>(tick_log_next_), tick_log_.end());
  v.insert(v.end(), tick_log_.begin(), tick_log_.begin() + static_cast<std::ptrdiff_t>(tick_log_next_));
  return v;
}

void Exporter::sampler_loop() {
  const bool rt = apply_rt(cfg_.rt_priority, "sampler", rt_threads_.get());
  // 1 us timer slack instead of the default 50 us: the tick starts on its deadline (t_late was
  // 70-90 us on MI355X boxes, profiles/r3_capacity.md); the sampler only sleeps in <= 50 ms
  // slices between ticks, so the extra precision costs nothing measurable
  prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
  const int64_t period = static_cast<int64_t>(cfg_.interval_s * 1e9);
  int64_t next = mono_ns() + period;
  next_tick_ns_->store(next, std::memory_order_release);
  while (running_) {
    int64_t now = mono_ns();
    if (now < next) {
      // sleep in short slices so stop() is prompt
      int64_t left = next - now;
      std::this_thread::sleep_for(std::chrono::nanoseconds(std::min<int64_t>(left, 50000000)));
      continue;
    }
    tick_deadline_ns_ = next;
    next_tick_ns_->store(next + period, std::memory_order_release);
    tick();
    tick_deadline_ns_ = 0;
    next += period;
    int64_t after = mono_ns();
    if (after > next) {
      // overran: skip missed slots, stay on the grid (deadline-based, unlike gpu.py:263)
      int64_t missed = (after - next) / period + 1;
      overruns_ += static_cast<uint64_t>(missed);
      next += missed * period;
      next_tick_ns_->store(next, std::memory_order_release);
    }
  }
  next_tick_ns_->store(0, std::memory_order_release);
  if (rt) rt_threads_->fetch_sub(1);
}

void Exporter::sample_devices(std::vector<DeviceSample>* out, std::vector<std::vector<ProcSample>>* procs,
                              double* procs_s, TickInfo* info) {
  int n = backend_->device_count();
  out->resize(n);
  procs->assign(n, {});
  // Link metrics (~1.2 ms per device: peer BDF, lane rate, max bandwidth — static while the link
  // state holds) are refreshed every `link_every` ticks, staggered so at most ceil(n / link_every)
  // devices pay it in one tick, and on the tick after a device's per-link status (read every tick
  // from the firmware table) changed. Per-tick link traffic and status never need this call.
  const uint64_t tk = ticks_.load();
  const bool links_ok = backend_->supports_links() && cfg_.link_every > 0;
  force_links_.resize(n, 0);
  links_read_.assign(n, 0);
  auto links_due = [&](int i) {
    const bool forced = force_links_[i] != 0;
    force_links_[i] = 0;
    const bool due =
        links_ok && (forced || tk == 0 || (tk + static_cast<uint64_t>(i)) % static_cast<uint64_t>(cfg_.link_every) == 0);
    links_read_[i] = due ? 1 : 0;
    if (due) info->link_refreshes++;
    return due;
  };
  // RAS: one full pass over the files every `ras_every` ticks (staggered per device), read as
  // `ras_slices` slices on consecutive ticks (1 = the whole pass on one tick: the fewest firmware
  // query bursts; more slices flatten the pass's tick-time spike). The first tick reads everything.
  const bool ras_ok = backend_->supports_ras() && cfg_.ras_every > 0;
  const int ras_period = std::max(1, cfg_.ras_every);
  const int ras_n = tk == 0 ? 1 : std::clamp(cfg_.ras_slices, 1, ras_period);
  auto ras_slice = [&](int i) {  // slice due for device i this tick, or -1
    if (!ras_ok) return -1;
    if (tk == 0) return 0;
    const int ph = static_cast<int>((tk + static_cast<uint64_t>(i)) % static_cast<uint64_t>(ras_period));
    return ph < ras_n ? ph : -1;
  };
  info->ras_full = ras_ok && ras_n == 1;
  int64_t proc_ns = 0;
  if (static_cast<int>(workers_.size()) != n) {
    // sequential: metrics table, (links), process list per device on the sampler thread
    const int64_t t_seq0 = mono_ns();
    for (int i = 0; i < n; ++i) {
      TraceRange tr("gpumon.sample_dev");
      backend_->sample(i, &(*out)[i]);
      if (links_due(i)) backend_->sample_links(i, &(*out)[i]);
      const int rs = ras_slice(i);
      if (rs >= 0 && (*out)[i].ok) {
        backend_->sample_ras(i, &(*out)[i], rs, ras_n);
        info->ras_reads++;
      }
      if (cfg_.processes && (*out)[i].ok) {
        const int64_t t = mono_ns();
        const bool ok = backend_->processes(i, &(*procs)[i]);
        (*out)[i].procs_read = ok ? 1 : backend_->supports_processes(i) ? -1 : 0;
        proc_ns += mono_ns() - t;
        for (auto& ps : (*procs)[i])
          if (has(ps.cu_occupancy)) {
            ps.occ_samples = 1;
            ps.occ_busy = ps.cu_occupancy > 0 ? 1 : 0;
          }
      }
    }
    *procs_s = proc_ns * 1e-9;
    info->t_device = (mono_ns() - t_seq0) * 1e-9;
    seq_maintain_ = cfg_.processes;  // tick() runs the upkeep after it published
    return;
  }
  const uint64_t id = ++tick_id_;
  const int64_t t0 = mono_ns();
  std::vector<char> asked(n, 0);
  for (int i = 0; i < n; ++i) {
    DevWorker& w = *workers_[i];
    std::lock_guard<std::mutex> g(w.mu);
    if (w.busy) continue;  // still inside an earlier (hung) call
    w.busy = w.pending = true;
    w.req = id;
    w.want_links = links_due(i);
    w.ras_slice = ras_slice(i);
    w.want_ras = w.ras_slice >= 0;
    w.ras_async = cfg_.ras_async && tk > 0;  // the first tick reads synchronously (complete first scrape)
    w.ras_n = ras_n;
    if (w.want_ras) info->ras_reads++;
    w.want_procs = cfg_.processes;
    w.started_ns = t0;
    asked[i] = 1;
    w.cv.notify_one();
  }
  const int64_t deadline = t0 + static_cast<int64_t>(cfg_.device_timeout_s * 1e9);
  auto all_done = [&] {
    for (int i = 0; i < n; ++i)
      if (asked[i] && workers_[i]->done.load(std::memory_order_acquire) != id) return false;
    return true;
  };
  {
    // Waits in <= 20 ms system_clock slices checked against the monotonic deadline: a steady_clock
    // wait_until compiles to pthread_cond_clockwait, which the toolchain's TSan does not intercept.
    std::unique_lock<std::mutex> lk(done_sig_->mu);
    while (!all_done()) {
      const int64_t left = deadline - mono_ns();
      if (left <= 0) break;
      done_sig_->cv.wait_until(lk, std::chrono::system_clock::now() +
                                       std::chrono::nanoseconds(std::min<int64_t>(left, 20'000'000)));
    }
  }
  for (int i = 0; i < n; ++i) {
    DevWorker& w = *workers_[i];
    std::lock_guard<std::mutex> g(w.mu);
    if (asked[i] && w.done.load(std::memory_order_acquire) == id) {
      (*out)[i] = std::move(w.sample);
      (*procs)[i] = std::move(w.procs);
      proc_ns += w.proc_ns;
      info->t_wake = std::max(info->t_wake, (w.picked_ns - w.started_ns) * 1e-9);
      info->t_device = std::max(info->t_device, w.device_ns * 1e-9);
      continue;
    }
    DeviceSample& s = (*out)[i];
    s.reset();
    s.host_mono_ns = mono_ns();
    s.host_wall_ns = wall_ns();
    s.ok = false;
    s.errors = 1;
    s.last_error = asked[i] ? "device call exceeded device_timeout_s" : "previous device call still running (hung)";
    std::lock_guard<std::mutex> g2(state_mu_);
    if (i < static_cast<int>(dev_timeouts_.size())) dev_timeouts_[i]++;
  }
  *procs_s = proc_ns * 1e-9;
}

void Exporter::set_device_mfma_util(std::map<int, double> v) {
  std::lock_guard<std::mutex> g(extra_mu_);
  mfma_util_ = std::move(v);
}

void Exporter::build_pod_rows(const std::vector<std::vector<ProcSample>>& procs,
                              const std::vector<DeviceSample>& samples, std::vector<PodRow>* rows) {
  rows->clear();
  // Exclusive use: the one process of a device whose waves were resident this interval (every
  // process counts, opted in or not). Its row carries the device's MFMA utilisation.
  std::map<int, double> mfma;
  {
    std::lock_guard<std::mutex> g(extra_mu_);
    mfma = mfma_util_;
  }
  // Shared vs exclusive (the reference dashboard's "(共享)" / "(独占)" columns, which counted the
  // pod_gpu rows of nvidia-smi's complete compute-apps list per GPU, gpu.py:111-116,190-219). A
  // non-helper process is a possible sharer of its device
  //  - while its waves were resident in any occupancy read of the tick (sub-samples included),
  //  - from the tick it ARRIVES holding VRAM, before any read could catch its waves (a 10 %-resident
  //    tenant is not read as absent in its first interval: VERDICT r2 #1), and
  //  - where residency is not observable on the device (no occupancy reads), while it holds VRAM;
  // and stops counting only after 5 ticks and mfma_exclusive_window_s without any of that (a
  // 10 %-resident tenant escapes 20 reads per tick 12 % of the time, the window's 100 reads 0.003 %).
  // The device is exclusive when one process is a sharer: its row carries the device MFMA util.
  std::vector<uint32_t> sole(procs.size(), 0);
  // The exporter's own on-device helper holds a GPU context on every device (PMC counter buffers)
  // and, with --probe, runs the K1 probe's waves: it is neither a workload row nor a sharer.
  const int helper_pid = ondevice_helper_pid();
  auto is_helper = [&](uint32_t pid) { return helper_pid > 0 && pid == static_cast<uint32_t>(helper_pid); };
  uint64_t helper_rows = 0;
  const uint64_t tick_no = ++pod_rows_built_;
  const int64_t now_ns = mono_ns();
  const int64_t window_ns = static_cast<int64_t>(std::max(0.0, cfg_.mfma_exclusive_window_s) * 1e9);
  if (last_active_.size() < procs.size()) last_active_.resize(procs.size());
  if (present_.size() < procs.size()) present_.resize(procs.size());
  if (sharing_source_.size() < procs.size()) sharing_source_.resize(procs.size());
  static const char* kSharingHelp =
      "Processes that may be using the GPU within the exclusivity window (5 ticks and "
      "mfma_exclusive_window_s): 0 idle, 1 exclusive, >1 shared. source=occupancy: waves resident in a KFD "
      "cu_occupancy read, or arrived holding VRAM; source=vram: every process holding VRAM (occupancy "
      "unreadable); source=allocations: pods allocated the GPU (process list off).";
  std::vector<ExtraSeries> sharing;
  // Peer contexts of multi-GPU processes (the usual 8-GPU tenant: torchrun with one rank per GPU,
  // each rank's runtime also opening every other GPU, RCCL importing peers' buffers). A (pid, GPU)
  // context is a peer context -- not a workload row, not a sharer -- when on that GPU it holds at
  // most peer_context_max_vram_mib, had no wave resident within the sharing window (where
  // occupancy is readable), and the same process has a workload context on ANOTHER GPU this tick
  // (more VRAM than that, or waves). The reference listed one row per compute app nvidia-smi
  // showed on a GPU (gpu.py:111-116,178,190-219): a rank appears on its own GPU only.
  if (last_waves_.size() < procs.size()) last_waves_.resize(procs.size());
  const double peer_floor = std::max(0.0, cfg_.peer_context_max_vram_mib) * 1048576.0;
  std::unordered_map<uint32_t, std::vector<int>> workload_devs;  // pid -> GPUs with a workload context
  std::vector<std::unordered_map<uint32_t, double>> vram_of(procs.size());  // (dev, pid) -> VRAM, contexts summed
  for (size_t d = 0; d < procs.size(); ++d) {
    auto& waves = last_waves_[d];
    for (const auto& p : procs[d]) {
      if (is_helper(p.pid)) continue;
      const double v = p.vram_bytes > 0 ? p.vram_bytes : (p.mem_bytes > 0 ? p.mem_bytes : 0.0);
      vram_of[d][p.pid] += v;
      if (p.occ_busy > 0 || p.cu_occupancy > 0) waves[p.pid] = {tick_no, now_ns};
    }
    for (auto it = waves.begin(); it != waves.end();) {  // forget pids past both windows
      if (tick_no - it->second.first >= 5 && now_ns - it->second.second >= window_ns) it = waves.erase(it);
      else ++it;
    }
    for (const auto& [pid, v] : vram_of[d])
      if (v > peer_floor || waves.count(pid)) workload_devs[pid].push_back(static_cast<int>(d));
  }
  auto is_peer = [&](size_t d, uint32_t pid) {
    if (peer_floor <= 0 || !cfg_.hide_empty_contexts) return false;
    if (last_waves_[d].count(pid)) return false;
    auto v = vram_of[d].find(pid);
    if (v != vram_of[d].end() && v->second > peer_floor) return false;
    auto w = workload_devs.find(pid);
    return w != workload_devs.end() &&
           std::any_of(w->second.begin(), w->second.end(), [&](int o) { return o != static_cast<int>(d); });
  };
  for (size_t d = 0; d < procs.size(); ++d) {
    if (!cfg_.processes) {  // no process list: the kubelet's allocations are what is known
      std::vector<std::pair<std::string, std::string>> pods;
      for (const auto& a : attr_->allocations())
        if (a.gpu_index == static_cast<int>(d) &&
            std::find(pods.begin(), pods.end(), std::make_pair(a.pod_namespace, a.pod_name)) == pods.end())
          pods.emplace_back(a.pod_namespace, a.pod_name);
      sharing.push_back({"gpu_active_processes", kSharingHelp, "gauge", static_cast<int>(d),
                         {{"source", "allocations"}}, static_cast<double>(pods.size())});
      continue;
    }
    auto& seen = last_active_[d];
    auto& present = present_[d];
    // residency is observable where occupancy can be read (also on a tick where no read has landed
    // yet for anyone: the first tick after start, a process that just arrived)
    const bool observable = std::any_of(procs[d].begin(), procs[d].end(),
                                        [](const ProcSample& p) { return p.occ_samples > 0; }) ||
                            (backend_ && backend_->supports_occupancy(static_cast<int>(d)));
    std::vector<uint32_t> active;  // distinct pids (one process may hold several KFD contexts)
    std::unordered_set<uint32_t> listed;
    for (const auto& p : procs[d]) {
      if (is_helper(p.pid) || is_peer(d, p.pid)) continue;
      const bool holds = p.vram_bytes > 0 || p.mem_bytes > 0;
      const bool waves = p.occ_busy > 0 || p.cu_occupancy > 0;
      if (holds || waves) listed.insert(p.pid);
      const bool arrived = holds && !present.count(p.pid);
      if ((waves || arrived || (!observable && holds)) && std::find(active.begin(), active.end(), p.pid) == active.end())
        active.push_back(p.pid);
    }
    // A tick whose device sample failed has no process list: it must not make every process look
    // like a new arrival on the next good tick, so the last list is kept.
    const bool listed_ok = d >= samples.size() || samples[d].ok;
    if (listed_ok) present.swap(listed);
    for (uint32_t pid : active) seen[pid] = {tick_no, now_ns};
    for (auto it = seen.begin(); it != seen.end();) {  // forget pids past both windows
      if (tick_no - it->second.first >= 5 && now_ns - it->second.second >= window_ns) it = seen.erase(it);
      else ++it;
    }
    if (active.size() == 1 && seen.size() == 1) sole[d] = active[0];
    std::string& src = sharing_source_[d];
    if (observable) src = "occupancy";
    else if (!procs[d].empty()) src = "vram";
    else if (src.empty()) src = backend_ && backend_->supports_occupancy(static_cast<int>(d)) ? "occupancy" : "vram";
    sharing.push_back({"gpu_active_processes", kSharingHelp, "gauge", static_cast<int>(d), {{"source", src}},
                       static_cast<double>(seen.size())});
  }
  for (const auto& dev_procs : procs)
    for (const auto& p : dev_procs) helper_rows += is_helper(p.pid) ? 1 : 0;
  if (helper_pid > 0)
    sharing.push_back({"gpumon_ondevice_helper_gpu_contexts",
                     "GPU contexts of the exporter's own on-device helper (PMC counting / K1 probe), left out of "
                     "pod_gpu rows and gpu_active_processes.",
                     "gauge", -1, {}, static_cast<double>(helper_rows)});
  set_extra("sharing", std::move(sharing));
  uint64_t hidden = 0, hidden_peer = 0;
  std::vector<uint32_t> alive;
  std::unordered_map<ProcKey, ProcPrev, ProcKeyHash> next_prev;
  // (ns, pod, container, dev) with an active process -> suppress the idle row for it
  std::vector<std::tuple<std::string, std::string, std::string, int>> active;
  for (size_t d = 0; d < procs.size(); ++d) {
    double dev_util = d < samples.size() ? samples[d].v[F_GFX_UTIL] : kNaN;
    // a held process list (the last good one, this tick's failed) carries no new engine time
    const bool held = d < samples.size() && samples[d].procs_held;
    // One row per (pid, device): duplicate entries (several KFD contexts of one process) are merged,
    // a duplicate series would make Prometheus reject the whole scrape.
    std::unordered_map<uint32_t, size_t> row_of_pid;
    for (const auto& p : procs[d]) {
      if (is_helper(p.pid)) continue;  // counted in gpumon_ondevice_helper_gpu_contexts
      auto dup = row_of_pid.find(p.pid);
      if (dup != row_of_pid.end()) {
        PodRow& r = (*rows)[dup->second];
        r.used_memory_bytes += has(p.vram_bytes) ? p.vram_bytes : 0;
        if (has(p.cu_occupancy)) r.cu_occupancy = has(r.cu_occupancy) ? r.cu_occupancy + p.cu_occupancy : p.cu_occupancy;
        continue;
      }
      // A KFD context that holds no VRAM and never had a wave resident this interval (a runtime
      // that only probed the device: rocminfo, amd-smi, an exporter's own HIP init) is not a GPU
      // workload; rows for it read as phantom 0-MiB processes. Counted, not exported.
      if (cfg_.hide_empty_contexts && !(p.vram_bytes > 0) && !(p.mem_bytes > 0) && !(p.cu_occupancy > 0) &&
          p.occ_busy == 0) {
        hidden++;
        continue;
      }
      if (is_peer(d, p.pid)) {  // a multi-GPU process's context on a GPU it does not work on (above)
        hidden_peer++;
        continue;
      }
      alive.push_back(p.pid);
      ProcIdentity id = attr_->resolve(p.pid);
      // per-process gfx util from engine_usage.gfx ns deltas
      double util = kNaN;
      int64_t now = mono_ns();
      if (p.has_gfx_ns) {
        ProcKey k{p.pid, static_cast<int>(d)};
        auto it = proc_prev_.find(k);
        if (held) {
          // the held list repeats the last reading: keep its baseline (the next good list's delta
          // then spans the whole gap) and its busy share, rather than a 0 % now and a spike later
          if (it != proc_prev_.end()) {
            next_prev[k] = it->second;
            util = it->second.util;
          }
        } else {
          if (it != proc_prev_.end() && it->second.starttime == id.starttime &&
              p.gfx_ns >= it->second.gfx_ns && now > it->second.t_ns)
            util = std::min(100.0, (p.gfx_ns - it->second.gfx_ns) * 100.0 / (now - it->second.t_ns));
          next_prev[k] = ProcPrev{p.gfx_ns, now, id.starttime, util};
        }
      }
      // HIP compute runs on KFD user queues, which DRM fdinfo engine time never sees: there the
      // process's busy % is the share of the interval's cu_occupancy reads that found its waves
      // resident (the per-process analogue of the device's gfx activity)
      if (!has(util) && p.occ_samples > 0) util = 100.0 * p.occ_busy / p.occ_samples;
      if (!id.opted_in) continue;
      PodRow r;
      r.dev = static_cast<int>(d);
      r.idle = false;
      r.pid = std::to_string(p.pid);
      std::string name = !p.name.empty() ? p.name : id.comm;
      // reference strips spaces from process names (gpu.py:203); keep them but escape properly
      r.procname = name.empty() ? "-" : name;
      r.pod_namespace = id.pod_namespace;
      r.pod_name = id.pod_name;
      r.container = id.container_name.empty() ? "-" : id.container_name;
      r.containerid = id.container_id.empty() ? "-" : id.container_id.substr(0, 12);
      r.user_name = id.user_name;
      r.extra_labels = std::move(id.extra_labels);
      r.used_memory_bytes = has(p.vram_bytes) ? p.vram_bytes : (has(p.mem_bytes) ? p.mem_bytes : 0);
      r.gpu_util = has(dev_util) ? dev_util : 0;
      r.proc_gfx_util = util;
      r.cu_occupancy = p.cu_occupancy;
      r.occ_samples = p.occ_samples;
      if (sole[d] == p.pid)
        if (auto m = mfma.find(static_cast<int>(d)); m != mfma.end()) r.mfma_util = m->second;
      // only a process attributed to a pod or container can stand in for its idle allocation row
      // (an unattributed host process reads "-" / "-" and must not swallow the allocation of a pod
      // whose name was unknown, also "-")
      if (r.pod_name != "-" || r.containerid != "-")
        active.emplace_back(r.pod_namespace, r.pod_name, r.container, r.dev);
      row_of_pid[p.pid] = rows->size();
      rows->push_back(std::move(r));
    }
  }
  proc_prev_.swap(next_prev);
  hidden_contexts_ = hidden;
  hidden_peer_contexts_ = hidden_peer;
  attr_->gc(alive);
  // Allocated-but-idle GPUs (reference gpu.py:220-253 via `docker exec nvidia-smi -L`; here the
  // kubelet PodResources allocation list pushed by the control plane).
  for (const auto& a : attr_->allocations()) {
    if (a.gpu_index < 0 || a.gpu_index >= static_cast<int>(procs.size())) continue;  // Q5
    if (!attr_->opted_in(a.labels)) continue;
    std::string ns = a.pod_namespace.empty() ? "-" : a.pod_namespace;
    std::string pod = a.pod_name.empty() ? "-" : a.pod_name;
    std::string ctr = a.container_name.empty() ? "-" : a.container_name;
    bool busy = false;
    for (const auto& t : active)
      if (std::get<0>(t) == ns && std::get<1>(t) == pod && std::get<3>(t) == a.gpu_index &&
          (std::get<2>(t) == ctr || std::get<2>(t) == "-")) {
        busy = true;
        break;
      }
    if (busy) continue;
    // the same (pod, container, GPU) listed twice must still be one series
    active.emplace_back(ns, pod, ctr, a.gpu_index);
    PodRow r;
    r.dev = a.gpu_index;
    r.idle = true;
    r.pod_namespace = ns;
    r.pod_name = pod;
    r.container = ctr;
    r.containerid = a.container_id.empty() ? "-" : a.container_id.substr(0, 12);
    r.user_name = !a.user_name.empty() ? a.user_name : attr_->derive_user(pod, a.labels);
    r.extra_labels = attr_->export_labels(a.labels);
    r.used_memory_bytes = 0;
    r.gpu_util = 0;
    rows->push_back(std::move(r));
  }
}

TickInfo Exporter::tick() {
  std::lock_guard<std::mutex> tl(tick_mu_);
  TraceRange trace_tick("gpumon.tick");
  TickInfo info;
  int64_t t0 = mono_ns();
  if (const int64_t dl = tick_deadline_ns_.load(); dl > 0) info.t_late = std::max<int64_t>(0, t0 - dl) * 1e-9;
  // this tick's results are built in place in the state it publishes (no copy in or out)
  auto next = std::make_shared<TickState>();
  std::vector<DeviceSample>& cur = next->samples;
  std::vector<DeviceRates>& rates = next->rates;
  std::vector<std::vector<ProcSample>>& procs = next->procs;
  std::vector<PodRow>& rows = next->rows;
  std::vector<size_t>& proc_counts = next->proc_counts;
  std::shared_ptr<const std::vector<DeviceStatic>> statics;
  bool up = ensure_backend();
  if (up) {
    statics = statics_ptr();
    int64_t ta = mono_ns();
    {
      TraceRange tr("gpumon.sample");
      sample_devices(&cur, &procs, &info.t_procs, &info);
    }
    int n = static_cast<int>(cur.size());
    info.t_sample = (mono_ns() - ta) * 1e-9;
    rates.resize(n);
    proc_counts.assign(n, 0);
    // the previous tick's samples and rates, by reference into its published state
    const std::shared_ptr<const TickState> prev_state = state_ptr();
    const std::vector<DeviceRates>& prev_rates = prev_state->rates;
    std::vector<const DeviceSample*> prev(std::min<size_t>(n, prev_state->samples.size()));
    for (size_t i = 0; i < prev.size(); ++i) prev[i] = &prev_state->samples[i];
    // A device whose previous tick failed is compared with its last good sample instead (if it is
    // recent): its interval rates then span the gap -- the accumulators make that exact -- rather
    // than going missing for the tick after every transient failure, and link identity and RAS
    // carry over the failed tick.
    if (static_cast<int>(last_ok_.size()) != n) last_ok_.assign(n, nullptr);
    const int64_t gap_ns = static_cast<int64_t>(std::max(5.0 * cfg_.interval_s, 5.0) * 1e9);
    for (int i = 0; i < static_cast<int>(prev.size()); ++i)
      if (!prev[i]->ok && last_ok_[i] && i < static_cast<int>(last_ok_[i]->samples.size())) {
        const DeviceSample& lo = last_ok_[i]->samples[i];
        if (lo.ok && cur[i].host_mono_ns - lo.host_mono_ns <= gap_ns) prev[i] = &lo;
      }
    std::vector<char> ok_now(n, 0), procs_good(n, 0);
    for (int i = 0; i < n; ++i) {
      DeviceSample& s = cur[i];
      // A link refresh counts only if the device answered AND the link-metrics read succeeded: a
      // timed-out or failed refresh keeps carrying the last identity and is retried next tick
      // (one failed refresh tick used to drop peer labels for up to link_every ticks).
      const bool asked_links = i < static_cast<int>(links_read_.size()) && links_read_[i];
      const bool refreshed = asked_links && s.ok && s.links_read == 1;
      if (asked_links && !refreshed && (!s.ok || s.links_read < 0) && i < static_cast<int>(force_links_.size()))
        force_links_[i] = 1;
      if (refreshed) {
        // pair link-metrics entries with table slots by their accumulators, then label the slots
        if (static_cast<int>(xgmi_maps_.size()) < n) xgmi_maps_.resize(n);
        xgmi_maps_[i].update(s);
        xgmi_maps_[i].apply(s.link_entries, &s);
      }
      if (i < static_cast<int>(prev.size())) {
        const DeviceSample& p = *prev[i];
        // keep link identity (peer bdf, max bw) between link refreshes -- but not on a tick that
        // re-read the links: an empty peer / unknown bandwidth then means the link lost them
        if (!refreshed)
          for (int k = 0; k < kMaxLinks; ++k) {
            if (s.links[k].peer_bdf.empty()) s.links[k].peer_bdf = p.links[k].peer_bdf;
            if (!has(s.links[k].max_bandwidth_gbps))
              s.links[k].max_bandwidth_gbps = p.links[k].max_bandwidth_gbps;
            if (s.links[k].link_type < 0) s.links[k].link_type = p.links[k].link_type;
          }
        if (!s.ras.valid && p.ras.valid && s.ok) s.ras = p.ras;  // between RAS refreshes
      }
      // A link's firmware status changed since the last SUCCESSFUL sample of this device (a failed
      // tick in between must not hide the change): re-read peer identity and bandwidth next tick.
      if (s.ok && i < static_cast<int>(force_links_.size())) {
        if (static_cast<int>(link_status_.size()) < n) link_status_.resize(n);
        auto& last = link_status_[i];
        if (!last.empty())
          for (int k = 0; k < kMaxLinks && k < static_cast<int>(last.size()); ++k)
            if (s.links[k].status >= 0 && last[k] >= 0 && s.links[k].status != last[k]) {
              force_links_[i] = 1;
              break;
            }
        last.assign(kMaxLinks, -1);
        for (int k = 0; k < kMaxLinks; ++k) last[k] = s.links[k].status;
      }
      // amdsmi_get_link_metrics lists 7 entries while the metrics table has 8 xGMI slots on
      // MI355X: a slot no link_metrics entry describes gets speed x width (38 Gb/s x 16 = 608 Gb/s,
      // the value link_metrics reports for every other link).
      const double lane = s.v[F_XGMI_LINK_SPEED], width = s.v[F_XGMI_LINK_WIDTH];
      for (int k = 0; k < s.n_links; ++k)
        if (s.links[k].status >= 0 && !has(s.links[k].max_bandwidth_gbps) && has(lane) && has(width))
          s.links[k].max_bandwidth_gbps = lane * width;
      if (static_cast<int>(last_fresh_ns_.size()) != n) last_fresh_ns_.assign(n, 0);
      if (i < static_cast<int>(prev.size())) {
        const DeviceSample& p = *prev[i];
        if (s.ok && p.ok && s.acc.firmware_ts && s.acc.firmware_ts == p.acc.firmware_ts) {
          s.fresh = false;
          stale_++;
        }
        // A repeated table (sampling faster than the firmware refresh) holds no new window: it
        // keeps the rates of the last one instead of reporting zero power / traffic over it --
        // but only while the table is younger than stale_hold_s. An older repeat means the SMU
        // stopped refreshing (hang, reset): the rates go invalid and gpu_metrics_table_frozen is 1
        // rather than exporting the last power / activity / xGMI rates forever.
        const bool young = last_fresh_ns_[i] > 0 && s.host_mono_ns - last_fresh_ns_[i] <= cfg_.stale_hold_s * 1e9;
        if (!s.fresh && young && i < static_cast<int>(prev_rates.size())) {
          rates[i] = prev_rates[i];
        } else if (!s.fresh) {
          rates[i] = DeviceRates{};
          frozen_++;
        } else {
          compute_rates(p, s, cfg_.rates, &rates[i]);
        }
      }
      if (s.ok && s.fresh && s.acc.firmware_ts) last_fresh_ns_[i] = s.host_mono_ns;
      samples_++;
      if (!s.ok || s.errors) {  // partial failures (one call failed, others answered) count too
        std::lock_guard<std::mutex> g(state_mu_);
        if (i < static_cast<int>(dev_errors_.size()))
          dev_errors_[i] += s.ok ? s.errors : std::max<uint32_t>(1, s.errors);
      }
      if (s.ok) {
        info.devices_ok++;
        ok_now[i] = 1;  // last_ok_[i] = this tick's state once it exists (below)
      }
      // A failed process list (a transient library or KFD error) keeps the last good list for up
      // to kProcHoldTicks ticks instead of publishing "no processes": every pod row of the GPU and
      // its sharing state would otherwise drop out for that tick. A device that never listed
      // successfully, or that cannot list at all, holds nothing.
      if (static_cast<int>(last_procs_.size()) != n) {
        last_procs_.assign(n, nullptr);
        proc_hold_.assign(n, -1);
      }
      if (s.procs_read > 0) {
        procs_good[i] = 1;  // last_procs_[i] = this tick's state (below)
        proc_hold_[i] = 0;
      } else if (s.procs_read < 0) {
        proc_failures_++;
        if (proc_hold_[i] >= 0 && proc_hold_[i] < kProcHoldTicks && last_procs_[i] &&
            i < static_cast<int>(last_procs_[i]->procs.size())) {
          procs[i] = last_procs_[i]->procs[i];
          // the held list's occupancy is the last good tick's: not a reading of this interval
          for (auto& hp : procs[i]) {
            hp.cu_occupancy = kNaN;
            hp.occ_samples = 0;
            hp.occ_busy = 0;
          }
          proc_hold_[i]++;
          s.procs_held = true;
        }
      }
      proc_counts[i] = procs[i].size();
      // device-level spatial occupancy: CUs holding any process's waves (every process, opted in or not)
      if (s.ok && cfg_.processes) {
        double cu = 0;
        bool any = false;
        for (const auto& p : procs[i])
          if (has(p.cu_occupancy)) {
            cu += p.cu_occupancy;
            any = true;
          }
        if (any || procs[i].empty()) s.v[F_CU_OCC] = cu;
      }
    }
    {
      // how far the xGMI peer labels rest on traffic evidence (xgmi_map.h)
      std::vector<ExtraSeries> xm;
      for (int i = 0; i < n && i < static_cast<int>(xgmi_maps_.size()); ++i) {
        const XgmiSlotMap& m = xgmi_maps_[i];
        if (m.empty()) continue;
        xm.push_back({"gpumon_xgmi_slot_map_mismatch",
                      "xGMI link-metrics entries whose peer was paired by traffic with a gpu_metrics slot other "
                      "than the entry's position (positional pairing would mislabel these peers).",
                      "gauge", i, {}, static_cast<double>(m.mismatched())});
        xm.push_back({"gpumon_xgmi_slot_map_verified",
                      "xGMI link-metrics entries with a peer whose gpu_metrics slot was confirmed by matching "
                      "accumulators (absolute or per-interval deltas).",
                      "gauge", i, {}, static_cast<double>(m.verified())});
        xm.push_back({"gpumon_xgmi_slot_map_unverified",
                      "xGMI link-metrics entries with a peer whose slot no traffic has confirmed yet (idle or "
                      "evenly loaded links): their peer label is positional or withheld.",
                      "gauge", i, {}, static_cast<double>(m.unverified())});
      }
      set_extra("xgmi_map", std::move(xm));
      // firmware-table freshness: how long since each table last advanced (host clock)
      std::vector<ExtraSeries> fz;
      for (int i = 0; i < n && i < static_cast<int>(last_fresh_ns_.size()); ++i) {
        const DeviceSample& s = cur[i];
        if (!s.ok || !s.acc.firmware_ts || last_fresh_ns_[i] <= 0) continue;
        const double age = std::max<int64_t>(0, s.host_mono_ns - last_fresh_ns_[i]) * 1e-9;
        fz.push_back({"gpu_metrics_table_age_seconds",
                      "Host seconds since the device's firmware metrics table (gpu_metrics) last advanced: 0 "
                      "on a fresh read; grows while the SMU serves the same table.",
                      "gauge", i, {}, age});
        fz.push_back({"gpu_metrics_table_frozen",
                      "1 while the firmware metrics table has not advanced for longer than stale_hold_s: "
                      "interval rates (power from energy, activity, xGMI) are withheld, instantaneous "
                      "values are the frozen table's.",
                      "gauge", i, {}, !s.fresh && age > cfg_.stale_hold_s ? 1.0 : 0.0});
      }
      set_extra("table_age", std::move(fz));
      std::vector<ExtraSeries> ph;
      for (int i = 0; i < n; ++i)
        if (cur[i].procs_read != 0)
          ph.push_back({"gpu_process_list_held",
                        "1 when this tick's process list failed and the GPU's last good list (at most 3 "
                        "ticks old) stands in for it.",
                        "gauge", i, {}, cur[i].procs_held ? 1.0 : 0.0});
      set_extra("procs_held", std::move(ph));
    }
    for (int i = 0; i < n; ++i) {
      if (ok_now[i]) last_ok_[i] = next;
      if (procs_good[i]) last_procs_[i] = next;
    }
    int64_t tb = mono_ns();
    {
      TraceRange tr("gpumon.attrib");
      build_pod_rows(procs, cur, &rows);
    }
    info.t_attrib = (mono_ns() - tb) * 1e-9;
    info.devices = n;
    // Whole-backend failure (driver reload, amdsmi lost its handles): re-initialise with backoff
    // instead of exporting gpu_up 0 forever (the reference crashed and relied on the kubelet).
    all_failed_ticks_ = (n > 0 && info.devices_ok == 0) ? all_failed_ticks_ + 1 : 0;
    if (cfg_.reinit_after > 0 && all_failed_ticks_ >= cfg_.reinit_after && workers_busy()) {
      // a worker is still inside a (hung) backend call: shutting the backend down under it is
      // unsafe; keep exporting gpu_up 0 until the call returns.
    } else if (cfg_.reinit_after > 0 && all_failed_ticks_ >= cfg_.reinit_after) {
      GPUMON_LOG(LogLevel::kWarn, "exporter",
                 "all " + std::to_string(n) + " GPU(s) failed " + std::to_string(all_failed_ticks_) +
                     " ticks in a row: re-initialising the backend");
      all_failed_ticks_ = 0;
      backend_up_ = false;
      reinits_++;
      next_init_ns_ = mono_ns();  // first retry immediately, then init_retry_s backoff
      backend_->shutdown();
    }
  }

  SelfStats self = self_stats();
  std::vector<ExtraSeries> extras;
  {
    std::lock_guard<std::mutex> g(extra_mu_);
    for (const auto& [src, v] : extras_) extras.insert(extras.end(), v.begin(), v.end());
  }
  self.pods_attributed = rows.size();
  RenderInput in;
  in.host = cfg_.host;
  static const std::vector<DeviceStatic> kNoStatics;
  static const std::vector<DeviceSample> kNoSamples;
  in.statics = up ? statics.get() : &kNoStatics;
  in.samples = up ? &cur : &kNoSamples;
  in.rates = &rates;
  in.pod_rows = &rows;
  in.proc_counts = &proc_counts;
  in.extras = &extras;
  in.self = &self;
  in.compat_families = cfg_.compat_families;
  in.extended_families = cfg_.extended_families;
  in.full_device_labels = cfg_.full_device_labels;
  in.metrics_include = &cfg_.metrics_include;
  in.metrics_exclude = &cfg_.metrics_exclude;
  auto snap = std::make_shared<Snapshot>();
  snap->gzip = cfg_.gzip;
  snap->body.reserve(std::max<size_t>(64 * 1024, last_body_bytes_ + last_body_bytes_ / 8));  // 8 GPUs: ~130 KB
  int64_t tr = mono_ns();
  {
    TraceRange trr("gpumon.render");
    render_prometheus(in, &snap->body);
  }
  info.t_render = (mono_ns() - tr) * 1e-9;
  snap->wall_ns = wall_ns();
  std::string influx;
  if (!cfg_.influx_url.empty() && cfg_.influx_every > 0 &&
      ticks_.load() % static_cast<uint64_t>(cfg_.influx_every) == 0) {
    render_influx(in, snap->wall_ns, cfg_.influx_extended, &influx, cfg_.influx_schema);
  }
  if (up) {
    std::shared_ptr<const TickState> published = next;
    std::lock_guard<std::mutex> g(state_mu_);
    state_.swap(published);  // the old state is released outside the lock (its last owner may be here)
  }
  info.pod_rows = rows.size();
  info.body_bytes = snap->body.size();
  last_body_bytes_ = snap->body.size();
  uint64_t s = seq_.load() + 1;
  snap->seq = s;
  // Publish the snapshot first (the tick's data is exported from here on); its gzip, when made by
  // this thread, follows the publish, off the sample-to-export path (0.1-0.4 ms for 1-8 GPUs at
  // level 1). A gzip scrape in between gets the identity body, which HTTP allows.
  std::shared_ptr<const Snapshot> published_snap = snap;
  std::shared_ptr<const Snapshot> prev_snap = store_.get();
  store_.publish(published_snap);
  ticks_++;
  last_tick_wall_ns_ = wall_ns();
  last_tick_mono_ns_ = mono_ns();
  info.duration_s = (mono_ns() - t0) * 1e-9;
  if (cfg_.gzip) {
    // This thread compresses the new snapshot (a) while scrapes keep asking for gzip (4 of the last
    // 8 snapshots), or (b) when a periodic gzip scraper's next scrape is predicted to land while
    // this snapshot is current (Prometheus at 15 s on a 1 Hz exporter: 1 compression per scrape,
    // made before the scrape arrives). Otherwise a scrape's first gzip request compresses its
    // snapshot itself (Snapshot::gzipped): correct, at the cost of that scrape's latency.
    gz_history_ = static_cast<uint8_t>((gz_history_ << 1) | (prev_snap && prev_snap->gzip_asked() ? 1 : 0));
    const bool frequent = __builtin_popcount(gz_history_) >= 4;
    bool predicted = false;
    const int64_t per = gz_period_ns_.load(std::memory_order_relaxed);
    const int64_t last = gz_last_scrape_ns_.load(std::memory_order_relaxed);
    if (!frequent && cfg_.interval_s > 0 && per > 0 && last > 0) {
      const int64_t now = mono_ns(), life = static_cast<int64_t>(cfg_.interval_s * 1e9);
      const int64_t slack = life / 10;
      int64_t next = last + per;
      // a scrape or two may have been missed (a restart, a slow network): keep the phase, but a
      // scraper silent for more than 3 periods is gone and nothing is predicted for it
      if (next < now - slack) next += ((now - slack - next) / per + 1) * per;
      predicted = next - last <= 4 * per && next >= now - slack && next <= now + life + slack;
    }
    if (frequent || predicted) {
      const int64_t tz = mono_ns();
      TraceRange trz("gpumon.gzip");
      snap->precompress();
      info.t_gzip = (mono_ns() - tz) * 1e-9;
      (frequent ? gz_eager_ : gz_predicted_)++;
    }
    if (prev_snap && prev_snap->compressed() && !prev_snap->gzip_asked()) gz_unused_++;
  }
  phase_ns_[0] += static_cast<uint64_t>(info.t_sample * 1e9);
  phase_ns_[1] += static_cast<uint64_t>(info.t_procs * 1e9);
  phase_ns_[2] += static_cast<uint64_t>(info.t_attrib * 1e9);
  phase_ns_[3] += static_cast<uint64_t>(info.t_render * 1e9);
  phase_ns_[4] += static_cast<uint64_t>(info.t_gzip * 1e9);
  sample_hist_.observe(info.duration_s);
  info.seq = s;
  {
    std::lock_guard<std::mutex> g(tick_log_mu_);
    if (tick_log_.size() < kTickLog) tick_log_.push_back(info);
    else tick_log_[tick_log_next_] = info;
    tick_log_next_ = (tick_log_next_ + 1) % kTickLog;
  }
  {
    std::lock_guard<std::mutex> g(seq_mu_);
    seq_ = s;
  }
  seq_cv_.notify_all();
  {
    SelfStats ps;
    read_process_stats(&ps);
    std::lock_guard<std::mutex> g(proc_stats_mu_);
    proc_stats_ = ps;
    proc_stats_valid_ = true;
  }
  if (seq_maintain_) {  // sequential sampling: no device worker to do it after the publish
    seq_maintain_ = false;
    for (int i = 0; i < backend_->device_count(); ++i) backend_->maintain(i);
  }
  if (!influx.empty()) {
    std::lock_guard<std::mutex> g(push_mu_);
    if (push_q_.size() >= 60) {
      push_q_.pop_front();
      influx_dropped_++;
    }
    push_q_.push_back(std::move(influx));
    push_cv_.notify_one();
  }
  return info;
}

bool Exporter::wait_for_seq(uint64_t want, double timeout_s) {
  std::unique_lock<std::mutex> lk(seq_mu_);
  // monotonic deadline in <= 100 ms system_clock slices (see podres_loop)
  const int64_t due = mono_ns() + static_cast<int64_t>(std::max(0.0, timeout_s) * 1e9);
  auto done = [&] { return seq_.load() >= want || !running_; };
  while (!done() && mono_ns() < due)
    seq_cv_.wait_until(lk, std::chrono::system_clock::now() +
                               std::chrono::nanoseconds(std::min<int64_t>(due - mono_ns(), 100'000'000)),
                       done);
  return seq_.load() >= want;
}

TlsOptions Exporter::influx_tls() const {
  TlsOptions t;
  t.ca_file = cfg_.influx_ca_file;
  t.insecure = cfg_.influx_tls_insecure;
  t.client_cert = cfg_.influx_client_cert;
  t.client_key = cfg_.influx_client_key;
  return t;
}

void Exporter::influx_loop() {
  // URL, token and TLS settings were checked by start() (check_push_config)
  const Url u = parse_url(cfg_.influx_url);
  HttpClient client(cfg_.influx_timeout_s);
  if (u.tls) {
    std::string terr;
    auto ctx = TlsContext::create(influx_tls(), &terr);
    if (!ctx) {  // checked at start: only a CA file removed since then lands here
      GPUMON_LOG(LogLevel::kError, "influx", "push disabled: " + terr);
      return;
    }
    if (cfg_.influx_tls_insecure)
      GPUMON_LOG(LogLevel::kWarn, "influx", "influx_tls_insecure: the server's certificate is NOT verified");
    client.set_tls(std::move(ctx));
  }
  const std::string headers = "Content-Type: text/plain; charset=utf-8\r\n" +
                              (!cfg_.influx_token.empty() ? "Authorization: Token " + cfg_.influx_token + "\r\n"
                                                          : u.auth_header);
  // A batch the server could not take for a transient reason (no connection, 5xx, 429) goes back
  // to the head of the queue and the push backs off (0.5 s doubling to 30 s), so an InfluxDB restart
  // loses nothing but what overflows the 60-batch queue; a 4xx other than 429 (a bad request, bad
  // credentials) would fail again and is dropped. Warnings: at most one per 10 s.
  int64_t backoff_ns = 0, retry_at = 0, last_warn = INT64_MIN / 2;
  uint64_t unlogged = 0;
  while (running_) {
    std::string body;
    {
      std::unique_lock<std::mutex> lk(push_mu_);
      const int64_t wait_ns = std::max<int64_t>(0, retry_at - mono_ns());
      // system_clock deadline: a steady_clock wait compiles to pthread_cond_clockwait, which the
      // toolchain's TSan does not intercept (it then reports the next lock as a double lock)
      push_cv_.wait_until(lk,
                          std::chrono::system_clock::now() +
                              std::chrono::nanoseconds(std::min<int64_t>(std::max<int64_t>(wait_ns, 1), 200'000'000)),
                          [&] { return !running_ || (!push_q_.empty() && mono_ns() >= retry_at); });
      if (!running_) break;
      if (push_q_.empty() || mono_ns() < retry_at) continue;
      body = std::move(push_q_.front());
      push_q_.pop_front();
    }
    std::string err, resp;
    int st = client.request("POST", u, body, headers, &resp, &err);
    if (st >= 200 && st < 300) {
      influx_ok_++;
      influx_up_ = 1;
      influx_last_ok_wall_ns_ = wall_ns();
      backoff_ns = 0;
      continue;
    }
    influx_fail_++;
    influx_up_ = 0;
    const bool transient = st < 0 || st >= 500 || st == 429;
    if (transient) {
      std::lock_guard<std::mutex> g(push_mu_);
      if (push_q_.size() < 60) push_q_.push_front(std::move(body));
      else influx_dropped_++;
      backoff_ns = std::clamp<int64_t>(backoff_ns * 2, 500'000'000, 30'000'000'000);
      retry_at = mono_ns() + backoff_ns;
    }
    const int64_t now = mono_ns();
    if (now - last_warn >= 10'000'000'000) {
      GPUMON_LOG(LogLevel::kWarn, "influx",
                 "push failed: " + (st < 0 ? err : ("HTTP " + std::to_string(st) + " " + resp.substr(0, 200))) +
                     (transient ? "; retrying in " + std::to_string(backoff_ns / 1'000'000) + " ms" : "; batch dropped") +
                     (unlogged ? " (" + std::to_string(unlogged) + " more failures since the last warning)" : ""));
      last_warn = now;
      unlogged = 0;
    } else {
      unlogged++;
    }
  }
}

bool Exporter::healthy() const {
  if (!running_) return false;
  double stale = cfg_.health_stale_s > 0 ? cfg_.health_stale_s
                                         : std::max(3.0 * cfg_.interval_s, 10.0);
  int64_t last = last_tick_mono_ns_.load();
  if (cfg_.interval_s <= 0) return last != 0;
  return last != 0 && (mono_ns() - last) * 1e-9 < stale;
}

namespace {

std::string url_decode(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] == '+') {
      o.push_back(' ');
    } else if (s[i] == '%' && i + 2 < s.size() && isxdigit(static_cast<unsigned char>(s[i + 1])) &&
               isxdigit(static_cast<unsigned char>(s[i + 2]))) {
      o.push_back(static_cast<char>(std::stoi(s.substr(i + 1, 2), nullptr, 16)));
      i += 2;
    } else {
      o.push_back(s[i]);
    }
  }
  return o;
}

// Bounds on a per-request filter: the globs come from any client that can reach the port, and a
// filter runs on an HTTP loop thread. Matching is O(glob x name) (glob_match), so these keep one
// request's work to ~32 globs x 128 chars x ~150 family names.
constexpr size_t kMaxFilterQuery = 8192, kMaxFilterGlobs = 32, kMaxGlobLen = 128;

// include=a,b&exclude=c (each repeatable): the family globs of a per-request filter.
// 1 = a filter, 0 = no filter keys, -1 = over the bounds above (*err says which).
int parse_filter_query(const std::string& q, std::vector<std::string>* inc, std::vector<std::string>* exc,
                       std::string* err) {
  if (q.size() > kMaxFilterQuery) {
    *err = "query longer than " + std::to_string(kMaxFilterQuery) + " bytes";
    return -1;
  }
  bool any = false;
  for (const auto& kv : split(q, '&')) {
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    const std::string k = url_decode(kv.substr(0, eq));
    std::vector<std::string>* dst = k == "include" ? inc : k == "exclude" ? exc : nullptr;
    if (!dst) continue;
    any = true;
    for (const auto& g : split(url_decode(kv.substr(eq + 1)), ',')) {
      if (g.empty()) continue;
      if (g.size() > kMaxGlobLen) {
        *err = "glob longer than " + std::to_string(kMaxGlobLen) + " bytes";
        return -1;
      }
      dst->push_back(g);
      if (inc->size() + exc->size() > kMaxFilterGlobs) {
        *err = "more than " + std::to_string(kMaxFilterGlobs) + " globs";
        return -1;
      }
    }
  }
  return any ? 1 : 0;
}

}  // namespace

std::shared_ptr<const Exporter::Filtered> Exporter::filtered(const Snapshot& s, const std::string& query, bool gzip) {
  {
    std::lock_guard<std::mutex> g(filter_mu_);
    if (filter_seq_ != s.seq) {
      filter_cache_.clear();
      filter_seq_ = s.seq;
    }
    auto it = filter_cache_.find(query);
    if (it != filter_cache_.end() && (!gzip || !it->second->body_gz.empty())) return it->second;
  }
  std::vector<std::string> inc, exc;
  std::string err;
  parse_filter_query(query, &inc, &exc, &err);  // handle_http validated it
  auto f = std::make_shared<Filtered>();
  filter_exposition(s.body, inc, exc, &f->body);
  if (gzip) gzip_compress(f->body, &f->body_gz, 1);
  std::lock_guard<std::mutex> g(filter_mu_);
  if (filter_seq_ == s.seq && (filter_cache_.size() < kFilterCache || filter_cache_.count(query)))
    filter_cache_[query] = f;
  return f;
}

void Exporter::handle_http(const HttpRequest& req, HttpResponse* resp) {
  if (req.path == "/metrics") {
    auto s = store_.get();
    if (!s) {
      resp->status = 503;
      resp->inline_body = "no sample yet\n";
      return;
    }
    resp->content_type = "text/plain; version=0.0.4; charset=utf-8";
    std::vector<std::string> inc, exc;
    std::string err;
    const int fq = req.query.empty() ? 0 : parse_filter_query(req.query, &inc, &exc, &err);
    if (fq < 0) {
      resp->status = 400;
      resp->inline_body = "bad family filter: " + err + "\n";
      return;
    }
    if (fq > 0) {
      // per-request family filter (e.g. a fast Prometheus job for node_gpu_* only)
      auto f = filtered(*s, req.query, req.accept_gzip && cfg_.gzip);
      if (req.accept_gzip && !f->body_gz.empty()) {
        resp->extra_headers = "Content-Encoding: gzip\r\n";
        resp->data = f->body_gz.data();
        resp->len = f->body_gz.size();
      } else {
        resp->data = f->body.data();
        resp->len = f->body.size();
      }
      resp->owner = f;
      return;
    }
    const bool fresh_gz = req.accept_gzip && s->gzip && !s->compressed();
    const std::string* gz = req.accept_gzip ? s->gzipped(true) : nullptr;
    if (fresh_gz && gz) gz_lazy_.fetch_add(1, std::memory_order_relaxed);
    if (req.accept_gzip && s->gzip) {
      // the gzip scrapers' cadence (EWMA of the spacing; bursts under 50 ms ignored) for the tick
      // thread's prediction above
      const int64_t now = mono_ns();
      const int64_t prev = gz_last_scrape_ns_.exchange(now, std::memory_order_relaxed);
      const int64_t d = prev > 0 ? now - prev : 0;
      if (d > 50'000'000) {
        const int64_t p = gz_period_ns_.load(std::memory_order_relaxed);
        gz_period_ns_.store(p > 0 && d < 8 * p ? (3 * p + d) / 4 : d, std::memory_order_relaxed);
      }
    }
    if (gz) {
      resp->extra_headers = "Content-Encoding: gzip\r\n";
      resp->data = gz->data();
      resp->len = gz->size();
    } else {
      resp->data = s->body.data();
      resp->len = s->body.size();
    }
    resp->owner = s;
    return;
  }
  if (req.path == "/healthz" || req.path == "/livez") {
    bool ok = healthy();
    resp->status = ok ? 200 : 503;
    resp->inline_body = ok ? "ok\n" : "sampler stalled\n";
    return;
  }
  if (req.path == "/readyz") {
    bool ok = ready() && backend_up_;
    resp->status = ok ? 200 : 503;
    resp->inline_body = ok ? "ready\n" : ("not ready: " + backend_error() + "\n");
    return;
  }
  if (req.path == "/" || req.path.empty()) {
    resp->content_type = "text/html; charset=utf-8";
    resp->inline_body =
        "<html><head><title>gpumon MI355X exporter</title></head><body><h1>gpumon</h1>"
        "<p><a href=\"/metrics\">/metrics</a> &middot; <a href=\"/healthz\">/healthz</a> &middot; "
        "<a href=\"/readyz\">/readyz</a></p></body></html>\n";
    return;
  }
  resp->status = 404;
  resp->inline_body = "not found\n";
}

void Exporter::set_extra(const std::string& source, std::vector<ExtraSeries> series) {
  std::lock_guard<std::mutex> g(extra_mu_);
  if (series.empty()) extras_.erase(source);
  else extras_[source] = std::move(series);
}

std::vector<DeviceStatic> Exporter::statics() const { return *statics_ptr(); }
std::vector<DeviceSample> Exporter::samples() const { return state_ptr()->samples; }
std::vector<int> Exporter::xcd_counts() const {
  const auto st = state_ptr();
  std::vector<int> out;
  out.reserve(st->samples.size());
  for (const auto& s : st->samples) out.push_back(s.n_xcd);
  return out;
}

std::vector<DeviceRates> Exporter::rates() const { return state_ptr()->rates; }
std::vector<PodRow> Exporter::pod_rows() const { return state_ptr()->rows; }

std::string Exporter::render_influx_now() {
  const auto st = statics_ptr();
  const auto state = state_ptr();
  RenderInput in;
  in.host = cfg_.host;
  in.statics = st.get();
  in.samples = &state->samples;
  in.pod_rows = &state->rows;
  std::string out;
  render_influx(in, wall_ns(), cfg_.influx_extended, &out, cfg_.influx_schema);
  return out;
}

// /proc/self based process collector (CPU, RSS, threads, fds, start time).
static void read_process_stats(SelfStats* s) {
  std::string st;
  if (read_file("/proc/self/stat", &st, 4096)) {
    size_t rp = st.rfind(')');
    if (rp != std::string::npos) {
      std::vector<std::string> f = split(std::string_view(st).substr(rp + 2), ' ');
      // after ") ": [0]=state ... [11]=utime [12]=stime [17]=num_threads [19]=starttime [21]=rss pages
      if (f.size() > 21) {
        const double hz = static_cast<double>(sysconf(_SC_CLK_TCK));
        const double page = static_cast<double>(sysconf(_SC_PAGESIZE));
        s->cpu_seconds = (atof(f[11].c_str()) + atof(f[12].c_str())) / hz;
        s->threads = atoi(f[17].c_str());
        s->rss_bytes = atof(f[21].c_str()) * page;
        std::string up;
        if (read_file("/proc/uptime", &up, 256)) {
          const double boot = wall_ns() * 1e-9 - atof(up.c_str());
          s->start_time_s = boot + atof(f[19].c_str()) / hz;
        }
      }
    }
  }
  if (DIR* d = opendir("/proc/self/fd")) {
    int n = 0;
    while (struct dirent* e = readdir(d))
      if (e->d_name[0] != '.') ++n;
    closedir(d);
    s->open_fds = n - 1;  // minus the directory handle itself
  }
}

SelfStats Exporter::self_stats() const {
  SelfStats s;
  s.version = cfg_.version;
  s.backend = backend_ ? backend_->name() : cfg_.backend;
  if (auto* a = dynamic_cast<AmdSmiBackend*>(backend_.get())) {
    s.backend_version = a->lib_version();
    s.fast_path_devices = a->fast_path_devices();
    s.fast_path_status = a->fast_path_status();
    a->kfd_file_stats(&s.kfd_files_open, &s.kfd_reads_cached);
  }
  if (auto* r = dynamic_cast<RocmSmiBackend*>(backend_.get())) s.backend_version = r->lib_version();
  s.backend_up = backend_up_;
  s.backend_reinits = reinits_;
  s.ticks = ticks_;
  s.samples = samples_;
  s.stale_samples = stale_;
  s.frozen_samples = frozen_;
  s.occupancy_reads = occ_reads_->load(std::memory_order_relaxed);
  s.occupancy_scan_failures = scan_failures_->load(std::memory_order_relaxed);
  s.process_list_failures = proc_failures_.load(std::memory_order_relaxed);
  s.hidden_contexts = hidden_contexts_.load();
  s.hidden_peer_contexts = hidden_peer_contexts_.load();
  s.rt_threads = rt_threads_->load();
  if (server_) {
    s.http_evicted = static_cast<int64_t>(server_->evicted());
    s.http_max_conns = static_cast<int64_t>(server_->max_conns() * static_cast<size_t>(std::max(1, cfg_.http_threads)));
  }
  if (cfg_.http_rt_priority > 0 && server_) {
    s.http_rt_loops = server_->rt_loops();
    s.http_rt_demotions = static_cast<int64_t>(server_->rt_demotions());
  }
  s.overruns = overruns_;
  s.last_tick_wall_s = last_tick_wall_ns_.load() * 1e-9;
  s.interval_s = cfg_.interval_s;
  sample_hist_.snapshot(&s.sample_hist.bounds, &s.sample_hist.counts, &s.sample_hist.count,
                        &s.sample_hist.sum);
  scrape_hist_.snapshot(&s.scrape_hist.bounds, &s.scrape_hist.counts, &s.scrape_hist.count,
                        &s.scrape_hist.sum);
  s.scrapes = s.scrape_hist.count;
  s.http_connections = server_ ? server_->connections() : 0;
  s.attribution_cache_hits = attr_->cache_hits();
  s.attribution_cache_misses = attr_->cache_misses();
  s.influx_ok = influx_ok_;
  s.influx_fail = influx_fail_;
  s.influx_dropped = influx_dropped_;
  s.influx_enabled = !cfg_.influx_url.empty();
  s.influx_up = influx_up_.load();
  s.influx_last_ok_wall_ns = influx_last_ok_wall_ns_.load();
  s.gzip_eager = gz_eager_.load(std::memory_order_relaxed);
  s.gzip_lazy = gz_lazy_.load(std::memory_order_relaxed);
  s.gzip_unused = gz_unused_.load(std::memory_order_relaxed);
  s.gzip_predicted = gz_predicted_.load(std::memory_order_relaxed);
  if (backend_)
    for (const auto& c : backend_->call_stats()) s.backend_calls.push_back({c.call, c.n, c.errors, c.seconds});
  {
    // the process's own CPU / RSS / threads / fds: read after each tick's publish (the /proc reads
    // took ~75 us, a third of a mock tick, on the sample -> export path), at most one tick old
    std::lock_guard<std::mutex> g(proc_stats_mu_);
    if (!proc_stats_valid_) {
      read_process_stats(&proc_stats_);
      proc_stats_valid_ = true;
    }
    s.cpu_seconds = proc_stats_.cpu_seconds;
    s.rss_bytes = proc_stats_.rss_bytes;
    s.start_time_s = proc_stats_.start_time_s;
    s.threads = proc_stats_.threads;
    s.open_fds = proc_stats_.open_fds;
  }
  {
    std::lock_guard<std::mutex> g(state_mu_);
    s.device_errors = dev_errors_;
    s.device_timeouts = dev_timeouts_;
    s.pods_attributed = state_->rows.size();
  }
  return s;
}

}  // namespace gpumon
