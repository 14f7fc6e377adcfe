// Per-device sampling workers (Exporter::start_workers / stop_workers and the worker loop). The
// tick that posts requests to them and collects the answers is Exporter::sample_devices
// (exporter.cpp).
#include "exporter_internal.h"

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>

#include "common.h"
#include "trace.h"

namespace gpumon {

// SCHED_FIFO for the calling thread (rt_priority); counted in `rt` while the thread lives.
bool apply_rt(int prio, const std::string& who, std::atomic<int>* rt) {
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

// Between ticks the worker sub-samples the KFD cu_occupancy of the processes its device had at
// the last tick, every occ_period_ns (interval / occ_samples): one read per tick is an instant
// (4.6 % of reads under a saturating burn land between two kernels and return 0, profiles/
// r2_kfd_occupancy.md); the tick's process rows carry the interval mean and the share of reads
// that found the process's waves resident.
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

}  // namespace gpumon
