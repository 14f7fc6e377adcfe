#include "exporter_internal.h"
#include "tls.h"

#include <pthread.h>
#include <sched.h>
#include <sys/prctl.h>

#include <dirent.h>
#include <unistd.h>

#include <algorithm>
#include <array>
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

// The exporter's tick, backend setup, Influx push and self stats. Split out: the device workers
// (dev_workers.cpp), pod_gpu attribution (pod_rows.cpp) and the HTTP endpoints (exporter_http.cpp).

static void read_process_stats(SelfStats* s);  // /proc/self figures (defined below)

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
  if (cfg_.serve_http && !cfg_.http_auth_token_file.empty()) {
    std::string e;
    auth_ = TokenAuth::create(cfg_.http_auth_token_file, &e);
    if (!auth_) {
      if (err) *err = e;
      return false;
    }
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
    if (!cfg_.tls_cert_file.empty() || !cfg_.tls_key_file.empty() || !cfg_.tls_client_ca_file.empty()) {
      auto tls = TlsServer::create(cfg_.tls_cert_file, cfg_.tls_key_file, cfg_.tls_client_ca_file, &e);
      if (!tls) {
        if (err) *err = e;
        server_.reset();
        return false;
      }
      server_->set_tls(std::move(tls));
    }
    if (!server_->start(&e)) {
      if (err) *err = e;
      server_.reset();
      return false;
    }
  }
  if (!cfg_.debug_listen.empty()) {
    std::string host, e;
    int port = 0;
    debug_server_ = parse_debug_listen(cfg_.debug_listen, &host, &port, &e)
                        ? std::make_unique<HttpServer>(
                              host, port, 1, [this](const HttpRequest& r, HttpResponse* w) { handle_debug(r, w); },
                              nullptr)
                        : nullptr;
    if (!debug_server_ || !debug_server_->start(&e)) {
      if (err) *err = e;
      debug_server_.reset();
      if (server_) server_->stop();
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
  // the introspection views read the /metrics server (its port, scrape durations): their loop
  // stops first. A /debug/wait in flight ended with running_ (above).
  if (debug_server_) debug_server_->stop();
  debug_server_.reset();
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
  info->dev.assign(n, TickDev{});
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
      const int64_t t_dev0 = mono_ns();
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
        info->dev[i].t_procs = (mono_ns() - t) * 1e-9;
        for (auto& ps : (*procs)[i])
          if (has(ps.cu_occupancy)) {
            ps.occ_samples = 1;
            ps.occ_busy = ps.cu_occupancy > 0 ? 1 : 0;
          }
      }
      info->dev[i].t_device = (mono_ns() - t_dev0) * 1e-9;
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
      info->dev[i].t_device = w.device_ns * 1e-9;
      info->dev[i].t_procs = w.proc_ns * 1e-9;
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
      // the firmware's PCIe bandwidth unit (rates.h RateConfig::pcie_bw_unit_bytes) -> bytes/s
      if (has(s.v[F_PCIE_BW_INST])) s.v[F_PCIE_BW_INST] *= cfg_.rates.pcie_bw_unit_bytes;
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
      build_pod_rows(procs, cur, &rows, &next->hidden);
    }
    info.t_attrib = (mono_ns() - tb) * 1e-9;
    info.devices = n;
    info.dev.resize(n);  // sample_devices sized it and set the per-device times
    for (int i = 0; i < n; ++i) {
      TickDev& d = info.dev[i];
      d.ok = cur[i].ok;
      d.fresh = cur[i].fresh;
      d.gfx_util = cur[i].v[F_GFX_UTIL];
      const DeviceRates& r = rates[i];
      d.rates_valid = r.valid;
      if (!r.valid) continue;
      double wr = 0, rd = 0;
      for (int k = 0; k < r.n_links; ++k) {
        if (has(r.xgmi_wr_Bps[k])) wr += r.xgmi_wr_Bps[k];
        if (has(r.xgmi_rd_Bps[k])) rd += r.xgmi_rd_Bps[k];
      }
      d.xgmi_wr_Bps = wr;
      d.xgmi_rd_Bps = rd;
      d.pcie_Bps = r.pcie_Bps;
    }
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
  // level 1). A gzip scrape in between compresses it itself, or waits for this thread's compression.
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
      // the margin around the predicted time: a tenth of a tick, widened to twice the scraper's
      // measured jitter (a loaded host, a jittery network), at most half a tick
      const int64_t slack =
          std::min(life / 2, std::max(life / 10, 2 * gz_jitter_ns_.load(std::memory_order_relaxed)));
      int64_t next = last + per;
      // a scrape or two may have been missed (a restart, a slow network): keep the phase, but a
      // scraper silent for more than 3 periods is gone and nothing is predicted for it
      if (next < now - slack) next += ((now - slack - next) / per + 1) * per;
      predicted = next - last <= 4 * per && next >= now - slack && next <= now + life + slack;
    }
    if (frequent || predicted) {
      const int64_t tz = mono_ns();
      TraceRange trz("gpumon.gzip");
      if (snap->precompress()) (frequent ? gz_eager_ : gz_predicted_)++;  // false: a scrape got there first
      info.t_gzip = (mono_ns() - tz) * 1e-9;
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
  block_sigpipe();  // an https push writes through OpenSSL's write() (common.h)
  // URL, token and TLS settings were checked by start() (check_push_config)
  const Url u = parse_url(cfg_.influx_url);
  HttpClient client(cfg_.influx_timeout_s);
  // the CA bundle and the client certificate / key rotate too (cert-manager): their files are
  // re-stamped every 30 s; a changed set is loaded and the connection reopened with it (a set that
  // does not load keeps the previous context and connection)
  const TlsOptions topt = influx_tls();
  auto stamps = [&] {
    return std::array<FileStamp, 3>{FileStamp::of(topt.ca_file), FileStamp::of(topt.client_cert),
                                    FileStamp::of(topt.client_key)};
  };
  std::array<FileStamp, 3> tls_stamps = stamps();
  const int64_t tls_period = tls_reload_period_ns(30'000'000'000LL);
  int64_t tls_check_at = mono_ns() + tls_period;
  if (u.tls) {
    std::string terr;
    auto ctx = TlsContext::create(topt, &terr);
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
  const std::string gz_headers = headers + "Content-Encoding: gzip\r\n";
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
    if (u.tls && (push_tls_check_now_.exchange(false) || mono_ns() >= tls_check_at)) {
      tls_check_at = mono_ns() + tls_period;
      if (const auto now = stamps(); now != tls_stamps) {
        tls_stamps = now;
        std::string terr;
        if (auto ctx = TlsContext::create(topt, &terr)) {
          client.set_tls(std::move(ctx));
          client.close_conn();  // the next push handshakes with the new files
          GPUMON_LOG(LogLevel::kInfo, "influx", "reloaded the push's TLS files");
        } else {
          GPUMON_LOG(LogLevel::kWarn, "influx", "the push's TLS files changed but do not load (keeping the previous ones): " + terr);
        }
      }
    }
    std::string err, resp, gz;
    // influx_gzip: the batch compressed (a requeued batch is kept plain and compressed again)
    const bool zipped = cfg_.influx_gzip && gzip_compress(body, &gz, 1);
    int st = client.request("POST", u, zipped ? gz : body, zipped ? gz_headers : headers, &resp, &err);
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

void Exporter::reload_tls() {
  push_tls_check_now_ = true;
  if (auth_) auth_->request_reload();
  if (server_)
    if (TlsServer* t = server_->tls_server()) t->request_reload();
}

bool Exporter::healthy() const {
  if (!running_) return false;
  double stale = cfg_.health_stale_s > 0 ? cfg_.health_stale_s
                                         : std::max(3.0 * cfg_.interval_s, 10.0);
  int64_t last = last_tick_mono_ns_.load();
  if (cfg_.interval_s <= 0) return last != 0;
  return last != 0 && (mono_ns() - last) * 1e-9 < stale;
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
  in.rates = &state->rates;
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
    if (const TlsServer* t = server_->tls_server()) {
      s.http_tls_failures = static_cast<int64_t>(server_->tls_failures());
      if (t->mutual()) s.http_tls_client_cert_refused = static_cast<int64_t>(mtls_refused_.load(std::memory_order_relaxed));
      s.http_tls_not_after = t->not_after();
      s.http_tls_reloads_ok = t->reloads_ok();
      s.http_tls_reloads_failed = t->reloads_failed();
    }
  }
  if (auth_) {
    for (int i = 0; i < 3; ++i) s.http_auth_failures_by[i] = auth_failures_[i].load(std::memory_order_relaxed);
    s.http_auth_failures = static_cast<int64_t>(s.http_auth_failures_by[0] + s.http_auth_failures_by[1] +
                                                s.http_auth_failures_by[2]);
    s.http_auth_reloads_ok = auth_->reloads_ok();
    s.http_auth_reloads_failed = auth_->reloads_failed();
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
