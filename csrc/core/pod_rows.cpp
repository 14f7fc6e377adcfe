// pod_gpu attribution: which (process, GPU) contexts become rows, their owners, and the idle
// allocation rows (Exporter::build_pod_rows, called once per tick from exporter.cpp).
#include "exporter_internal.h"

#include <algorithm>
#include <cmath>
#include <unordered_set>

#include "common.h"
#include "ondevice.h"

namespace gpumon {

void Exporter::build_pod_rows(const std::vector<std::vector<ProcSample>>& procs,
                              const std::vector<DeviceSample>& samples, std::vector<PodRow>* rows,
                              std::vector<HiddenCtx>* hidden_out) {
  rows->clear();
  if (hidden_out) hidden_out->clear();
  auto hide = [&](size_t d, uint32_t pid, const char* why) {
    if (hidden_out) hidden_out->push_back({static_cast<int>(d), pid, why});
  };
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
  // context is a peer context -- not a workload row, not a sharer -- when the process never
  // submitted work to that GPU and has a workload on ANOTHER GPU this tick:
  //  * where KFD lists the process's queues (sysfs fast path): no hardware queue on that GPU and
  //    no wave resident within the sharing window, whatever VRAM it holds there. A TP / PP process
  //    that computes on a second GPU holds queues there and keeps that row however small its shard
  //    (measured on MI355X: an allocate-only context has no queue, one kernel or copy creates them;
  //    profiles/r6_kfd_queues.md);
  //  * elsewhere (the queue list unreadable, libamd_smi process lists): at most
  //    peer_context_max_vram_mib there and no wave within the window.
  // A workload context is one with queues or waves, or (queues unknown) more VRAM than that. The
  // reference listed one row per compute app nvidia-smi showed on a GPU (gpu.py:111-116,178,190-219):
  // a rank appears on its own GPU only. peer_context_max_vram_mib 0 turns the rule off.
  if (last_waves_.size() < procs.size()) last_waves_.resize(procs.size());
  const double peer_floor = std::max(0.0, cfg_.peer_context_max_vram_mib) * 1048576.0;
  std::unordered_map<uint32_t, std::vector<int>> workload_devs;  // pid -> GPUs with a workload context
  std::vector<std::unordered_map<uint32_t, double>> vram_of(procs.size());  // (dev, pid) -> VRAM, contexts summed
  std::vector<std::unordered_map<uint32_t, int>> queues_of(procs.size());   // (dev, pid) -> queues (-1 unknown)
  for (size_t d = 0; d < procs.size(); ++d) {
    auto& waves = last_waves_[d];
    for (const auto& p : procs[d]) {
      if (is_helper(p.pid)) continue;
      const double v = p.vram_bytes > 0 ? p.vram_bytes : (p.mem_bytes > 0 ? p.mem_bytes : 0.0);
      vram_of[d][p.pid] += v;
      auto q = queues_of[d].emplace(p.pid, p.queues);
      if (!q.second && p.queues >= 0) q.first->second = std::max(q.first->second, 0) + p.queues;
      if (p.occ_busy > 0 || p.cu_occupancy > 0) waves[p.pid] = {tick_no, now_ns};
    }
    for (auto it = waves.begin(); it != waves.end();) {  // forget pids past both windows
      if (tick_no - it->second.first >= 5 && now_ns - it->second.second >= window_ns) it = waves.erase(it);
      else ++it;
    }
    for (const auto& [pid, v] : vram_of[d]) {
      const int q = queues_of[d][pid];
      if (waves.count(pid) || q > 0 || (q < 0 && v > peer_floor)) workload_devs[pid].push_back(static_cast<int>(d));
    }
  }
  auto is_peer = [&](size_t d, uint32_t pid) {
    if (peer_floor <= 0 || !cfg_.hide_empty_contexts) return false;
    if (last_waves_[d].count(pid)) return false;
    auto q = queues_of[d].find(pid);
    const int queues = q == queues_of[d].end() ? -1 : q->second;
    if (queues > 0) return false;  // it submitted work to this GPU
    if (queues < 0) {              // no queue list: the VRAM threshold
      auto v = vram_of[d].find(pid);
      if (v != vram_of[d].end() && v->second > peer_floor) return false;
    }
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
      if (is_helper(p.pid)) {  // counted in gpumon_ondevice_helper_gpu_contexts
        hide(d, p.pid, "helper");
        continue;
      }
      auto dup = row_of_pid.find(p.pid);
      if (dup != row_of_pid.end()) {
        PodRow& r = (*rows)[dup->second];
        r.used_memory_bytes += has(p.vram_bytes) ? p.vram_bytes : 0;
        if (p.queues >= 0) r.queues = std::max(r.queues, 0) + p.queues;
        if (has(p.cu_occupancy)) r.cu_occupancy = has(r.cu_occupancy) ? r.cu_occupancy + p.cu_occupancy : p.cu_occupancy;
        continue;
      }
      // A KFD context that holds no VRAM and never had a wave resident this interval (a runtime
      // that only probed the device: rocminfo, amd-smi, an exporter's own HIP init) is not a GPU
      // workload; rows for it read as phantom 0-MiB processes. Counted, not exported.
      if (cfg_.hide_empty_contexts && !(p.vram_bytes > 0) && !(p.mem_bytes > 0) && !(p.cu_occupancy > 0) &&
          p.occ_busy == 0) {
        hidden++;
        hide(d, p.pid, "empty");
        continue;
      }
      if (is_peer(d, p.pid)) {  // a multi-GPU process's context on a GPU it does not work on (above)
        hidden_peer++;
        hide(d, p.pid, "peer");
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
      if (!id.opted_in) {
        hide(d, p.pid, "not opted in");
        continue;
      }
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
      r.queues = p.queues;
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

}  // namespace gpumon
