// Kubernetes / container-runtime metadata for the exporter: the native pollers that feed the
// attributor (csrc/core/attribution.h) its container table and GPU allocations.
//   * kubelet PodResources List() (grpc_lite.h)  -> allocations (idle pod_gpu rows)
//   * CRI ListContainers / ListPodSandbox          -> pod name / namespace / labels per container
//   * Docker Engine API (docker_lite.h, opt-in)    -> the same on plain-Docker nodes + GPU devices
//   * kubelet-written files (kubelet_files.h)      -> both, socket-free, for a non-root exporter
// Reference counterpart: `docker ps` / `docker inspect` / `docker top` / `docker exec nvidia-smi -L`
// over the host's docker.sock (/root/reference/gpu.py:86-103,177,221-223).
#include <algorithm>
#include <cstring>
#include <unordered_map>
#include <unordered_set>

#include "common.h"
#include "docker_lite.h"
#include "exporter.h"
#include "grpc_lite.h"
#include "kubelet_files.h"

namespace gpumon {

// ---------------------------------------------------------------------------------------------
// Native PodResources poller (standalone binary): kubelet List() -> Allocation table.
// ---------------------------------------------------------------------------------------------
namespace {
std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
  return s;
}
}  // namespace

// Device-plugin device ID -> exporter device index (-1 unknown). The AMD device plugin uses PCI
// addresses; UUIDs, hip ids and DRM node names are accepted too (tests/oracles/attribution/plane.py).
int match_device_id(const std::string& raw, const std::vector<DeviceStatic>& st) {
  std::string d = lower(std::string(trim(raw)));
  // DRA forms: CDI name "amd.com/gpu=gpu-0" (part after '='), "gpu-N" (hip id), dashed PCI address
  // "gpu-0000-26-00-0" / "pci-0000-26-00-0" / "0000-26-00-0"
  if (auto eq = d.find('='); eq != std::string::npos) d = d.substr(eq + 1);
  {
    std::string x = d;
    if (starts_with(x, "gpu-") || starts_with(x, "pci-")) x = x.substr(4);
    auto hex = [](char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'); };
    if (x.size() == 12 && x[4] == '-' && x[7] == '-' && x[10] == '-' && x[11] >= '0' && x[11] <= '7' &&
        std::all_of(x.begin(), x.begin() + 4, hex) && hex(x[5]) && hex(x[6]) && hex(x[8]) && hex(x[9]))
      d = x.substr(0, 4) + ":" + x.substr(5, 2) + ":" + x.substr(8, 2) + "." + x.substr(11);
    else if (starts_with(d, "gpu-") && d.size() > 4 &&
             std::all_of(d.begin() + 4, d.end(), [](char c) { return c >= '0' && c <= '9'; }))
      d = d.substr(4);
  }
  if (d.empty()) return -1;
  for (const auto& s : st) {
    const std::string bdf = lower(s.bdf);
    if (!bdf.empty()) {
      if (d == bdf) return s.index;
      if (d.find(':') != std::string::npos && ends_with(bdf, d)) return s.index;  // without domain
    }
    const std::string uuid = lower(s.uuid);
    if (!uuid.empty() && (d == uuid || d == "gpu-" + uuid)) return s.index;
  }
  for (const auto& s : st) {
    const bool digits = std::all_of(d.begin(), d.end(), [](char c) { return c >= '0' && c <= '9'; });
    if (digits && std::to_string(s.hip_id) == d) return s.index;
    if (starts_with(d, "card") && d.substr(4) == std::to_string(s.drm_card)) return s.index;
    if (starts_with(d, "renderd") && d.substr(7) == std::to_string(s.drm_render)) return s.index;
  }
  return -1;
}

bool Exporter::podres_poll_once() {
  std::vector<PodDeviceRow> rows;
  std::string err;
  const int64_t t0 = mono_ns();
  GrpcStatus gst;
  const bool ok = podresources_list(cfg_.pod_resources_socket, cfg_.pod_resources_prefix, &rows, &err, 3000,
                                    cfg_.pod_resources_dra_drivers, &gst);
  const double dt = (mono_ns() - t0) * 1e-9;
  std::vector<DeviceStatic> st;
  {
    std::lock_guard<std::mutex> g(state_mu_);
    st = *statics_;
  }
  size_t unknown = 0;
  if (ok) {
    std::vector<Allocation> allocs;
    for (const auto& r : rows) {
      const int idx = match_device_id(r.device_id, st);
      if (idx < 0) {
        unknown++;  // Q5: the reference emitted gpu_id=None for these (gpu.py:226)
        continue;
      }
      Allocation a;
      a.pod_namespace = r.pod_namespace;
      a.pod_name = r.pod_name;
      a.container_name = r.container_name;
      a.gpu_index = idx;
      {
        // enrich from CRI (container id, pod uid, labels for the opt-in gate and user label)
        std::lock_guard<std::mutex> g(podres_mu_);
        const auto it = native_meta_.find(r.pod_namespace + "/" + r.pod_name + "/" + r.container_name);
        if (it != native_meta_.end()) {
          a.container_id = it->second.container_id;
          a.pod_uid = it->second.pod_uid;
          a.labels = it->second.labels;
        }
      }
      allocs.push_back(std::move(a));
    }
    {
      std::lock_guard<std::mutex> g(meta_mu_);
      podres_allocs_ = std::move(allocs);
    }
    publish_allocations();
  } else {
    GPUMON_LOG(LogLevel::kWarn, "podresources", "List() failed: " + err);
  }
  std::vector<ExtraSeries> ex;
  ex.push_back({"gpumon_podresources_up", "1 if the last kubelet PodResources List() succeeded.", "gauge", -1, {},
                ok ? 1.0 : 0.0});
  ex.push_back({"gpumon_podresources_unknown_devices", "Allocated device IDs that match no local GPU.", "gauge",
                -1, {}, static_cast<double>(unknown)});
  ex.push_back({"gpumon_podresources_list_seconds", "Duration of the last PodResources List() call.", "gauge", -1,
                {}, dt});
  ex.push_back({"gpumon_podresources_grpc_status",
                "grpc-status of the last PodResources List() (0 OK, 7 PERMISSION_DENIED, 12 UNIMPLEMENTED, ...; "
                "-1 = no status: transport failure).",
                "gauge", -1, {}, static_cast<double>(gst.code)});
  set_extra("podresources_native", std::move(ex));
  return ok;
}

void Exporter::podres_loop() {
  std::unique_lock<std::mutex> lk(podres_mu_);
  while (running_) {
    // Monotonic deadline, waited in <= 1 s system_clock slices: TSan does not intercept the
    // pthread_cond_clockwait a steady_clock wait compiles to, and a single system_clock wait
    // would stretch by however far the wall clock is stepped back meanwhile.
    const int64_t due = mono_ns() + static_cast<int64_t>(std::max(0.5, cfg_.pod_resources_refresh_s) * 1e9);
    while (running_ && mono_ns() < due)
      podres_cv_.wait_until(lk, std::chrono::system_clock::now() +
                                    std::chrono::nanoseconds(std::min<int64_t>(due - mono_ns(), 1'000'000'000)),
                            [&] { return !running_.load(); });
    if (!running_) break;
    lk.unlock();
    if (!cfg_.cri_socket.empty()) cri_poll_once();
    if (!cfg_.docker_socket.empty()) docker_poll_once();
    if (!cfg_.pod_log_root.empty() || !cfg_.device_checkpoint.empty()) files_poll_once();
    if (!cfg_.pod_resources_socket.empty()) podres_poll_once();
    lk.lock();
  }
}

// CRI containers + sandboxes -> ContainerMeta (same merge as tests/oracles/attribution/plane.py: pod
// annotations < pod labels < container annotations < container labels).
bool Exporter::cri_poll_once() {
  std::vector<CriContainer> cs;
  std::vector<CriSandbox> sbs;
  std::string err;
  const int64_t t0 = mono_ns();
  GrpcStatus gst;
  const bool ok = cri_list(cfg_.cri_socket, &cs, &sbs, &err, 3000, &gst);
  const double dt = (mono_ns() - t0) * 1e-9;
  if (ok) {
    std::unordered_map<std::string, const CriSandbox*> by_id;
    for (const auto& s : sbs) by_id[s.id] = &s;
    std::vector<ContainerMeta> metas;
    metas.reserve(cs.size());
    for (const auto& c : cs) {
      const auto it = by_id.find(c.sandbox_id);
      const CriSandbox* sb = it == by_id.end() ? nullptr : it->second;
      ContainerMeta m;
      m.container_id = c.id;
      if (sb) {
        m.labels.insert(sb->annotations.begin(), sb->annotations.end());
        for (const auto& kv : sb->labels) m.labels[kv.first] = kv.second;
      }
      for (const auto& kv : c.annotations) m.labels[kv.first] = kv.second;
      for (const auto& kv : c.labels) m.labels[kv.first] = kv.second;
      auto lab = [&](const char* k, const std::string& dflt) {
        const auto l = c.labels.find(k);
        return l != c.labels.end() && !l->second.empty() ? l->second : dflt;
      };
      m.container_name = lab("io.kubernetes.container.name", c.name);
      m.pod_name = lab("io.kubernetes.pod.name", sb ? sb->name : "");
      m.pod_namespace = lab("io.kubernetes.pod.namespace", sb ? sb->pod_namespace : "");
      m.pod_uid = lab("io.kubernetes.pod.uid", sb ? sb->uid : "");
      metas.push_back(std::move(m));
    }
    {
      std::lock_guard<std::mutex> g(meta_mu_);
      cri_metas_ = std::move(metas);
    }
    publish_container_meta();
  } else {
    GPUMON_LOG(LogLevel::kWarn, "cri", "ListContainers/ListPodSandbox failed: " + err);
  }
  std::vector<ExtraSeries> ex;
  ex.push_back({"gpumon_cri_up", "1 if the last CRI ListContainers/ListPodSandbox succeeded.", "gauge", -1, {},
                ok ? 1.0 : 0.0});
  ex.push_back({"gpumon_cri_containers", "Containers known from the CRI runtime.", "gauge", -1, {},
                static_cast<double>(cs.size())});
  ex.push_back({"gpumon_cri_list_seconds", "Duration of the last CRI listing.", "gauge", -1, {}, dt});
  ex.push_back({"gpumon_cri_grpc_status",
                "grpc-status of the last CRI call (0 OK, 12 UNIMPLEMENTED after both runtime.v1 and v1alpha2, ...; "
                "-1 = no status: transport failure).",
                "gauge", -1, {}, static_cast<double>(gst.code)});
  set_extra("cri_native", std::move(ex));
  return ok;
}

// CRI metadata first; Docker listings add the containers no CRI runtime reported (plain-Docker
// nodes, or dockershim-era nodes where both are configured). Empty pod names (non-k8s containers)
// never enter the PodResources join.
void Exporter::publish_container_meta() {
  std::vector<ContainerMeta> all;
  {
    std::lock_guard<std::mutex> g(meta_mu_);
    all = cri_metas_;
    std::unordered_set<std::string> seen;
    for (const auto& m : all) seen.insert(m.container_id);
    for (const auto& m : docker_metas_)
      if (seen.insert(m.container_id).second) all.push_back(m);
    for (const auto& m : files_metas_)
      if (seen.insert(m.container_id).second) all.push_back(m);
  }
  {
    std::lock_guard<std::mutex> g(podres_mu_);
    native_meta_.clear();
    for (const auto& m : all)
      if (!m.pod_name.empty()) native_meta_[m.pod_namespace + "/" + m.pod_name + "/" + m.container_name] = m;
  }
  attr_->set_container_meta(std::move(all));
}

// Docker Engine GET /containers/json -> ContainerMeta. The reference's `docker inspect` read the
// same Config.Labels (/root/reference/gpu.py:86-88,184-195): io.kubernetes.* on dockershim-managed
// containers, user labels (e.g. the `mlgpu` opt-in) on any container.
bool Exporter::docker_poll_once() {
  std::vector<DockerContainer> cs;
  std::string err;
  int http = -1;
  const int64_t t0 = mono_ns();
  const bool ok = docker_list(cfg_.docker_socket, &cs, &err, 3000, &http);
  uint64_t inspect_errors = 0;
  const double dt = (mono_ns() - t0) * 1e-9;
  if (ok) {
    std::vector<ContainerMeta> metas;
    metas.reserve(cs.size());
    for (auto& c : cs) {
      ContainerMeta m;
      m.container_id = c.id;
      auto lab = [&](const char* k, const std::string& dflt) {
        const auto l = c.labels.find(k);
        return l != c.labels.end() && !l->second.empty() ? l->second : dflt;
      };
      m.container_name = lab("io.kubernetes.container.name", c.name);
      m.pod_name = lab("io.kubernetes.pod.name", "");
      m.pod_namespace = lab("io.kubernetes.pod.namespace", "");
      m.pod_uid = lab("io.kubernetes.pod.uid", "");
      m.labels = std::move(c.labels);
      metas.push_back(std::move(m));
    }
    // which GPUs each container holds: one inspect per container the first time it is seen
    std::vector<DeviceStatic> st;
    {
      std::lock_guard<std::mutex> g(state_mu_);
      st = *statics_;
    }
    std::unordered_map<std::string, DockerInspect> seen;
    std::unordered_map<std::string, std::vector<int>> gpus;
    int inspected = 0;
    for (const auto& m : metas) {
      auto it = docker_inspects_.find(m.container_id);
      if (it != docker_inspects_.end()) {
        gpus.emplace(m.container_id, docker_container_gpus(it->second, st));
        seen.emplace(m.container_id, std::move(it->second));
        continue;
      }
      if (inspected >= 64) continue;  // bounded per refresh; the rest next time
      DockerInspect di;
      std::string ierr;
      ++inspected;
      if (docker_inspect(cfg_.docker_socket, m.container_id, &di, &ierr, 3000)) {
        gpus.emplace(m.container_id, docker_container_gpus(di, st));
        seen.emplace(m.container_id, std::move(di));
      } else {
        inspect_errors++;
        GPUMON_LOG(LogLevel::kDebug, "docker", "inspect " + m.container_id.substr(0, 12) + ": " + ierr);
      }
    }
    std::vector<Allocation> allocs;
    for (const auto& m : metas) {
      const auto it = gpus.find(m.container_id);
      if (it == gpus.end()) continue;
      for (int idx : it->second) {
        Allocation a;
        a.pod_namespace = m.pod_namespace;
        a.pod_name = m.pod_name;
        a.container_name = m.container_name;
        a.container_id = m.container_id;
        a.pod_uid = m.pod_uid;
        a.labels = m.labels;
        a.gpu_index = idx;
        allocs.push_back(std::move(a));
      }
    }
    docker_inspects_.swap(seen);  // forgets containers that are gone
    {
      std::lock_guard<std::mutex> g(meta_mu_);
      docker_metas_ = std::move(metas);
      docker_allocs_ = std::move(allocs);
    }
    publish_container_meta();
    publish_allocations();
  } else {
    GPUMON_LOG(LogLevel::kWarn, "docker", "GET /containers/json failed: " + err);
  }
  std::vector<ExtraSeries> ex;
  ex.push_back({"gpumon_docker_up", "1 if the last Docker Engine GET /containers/json succeeded.", "gauge", -1, {},
                ok ? 1.0 : 0.0});
  ex.push_back({"gpumon_docker_containers", "Containers known from the Docker Engine API.", "gauge", -1, {},
                static_cast<double>(cs.size())});
  ex.push_back({"gpumon_docker_list_seconds", "Duration of the last Docker Engine listing.", "gauge", -1, {}, dt});
  ex.push_back({"gpumon_docker_inspect_errors", "Container inspects that failed in the last Docker refresh.", "gauge",
                -1, {}, static_cast<double>(inspect_errors)});
  ex.push_back({"gpumon_docker_http_status",
                "HTTP status of the last Docker Engine listing (-1 = transport failure).", "gauge", -1, {},
                static_cast<double>(http)});
  set_extra("docker_native", std::move(ex));
  return ok;
}

// Kubelet-written files (kubelet_files.h): the log tree names every container on the node; the
// device-plugin checkpoint lists the GPUs each (pod uid, container) was given. A checkpoint entry
// of a pod without a log directory (gone from the node) is dropped, and so is one whose container
// has no live process (a Completed / Failed pod the kubelet has not deleted: its checkpoint entry
// and log directory stay until then) -- where the process scan can tell.
bool Exporter::files_poll_once() {
  std::vector<ContainerMeta> metas;
  std::string err;
  bool logs_ok = false, ckpt_ok = false;
  if (!cfg_.pod_log_root.empty()) {
    logs_ok = kubelet_log_metadata(cfg_.pod_log_root, &metas, &err);
    if (!logs_ok) GPUMON_LOG(LogLevel::kWarn, "kubelet-files", "pod log tree: " + err);
  }
  std::vector<Allocation> allocs;
  std::vector<std::vector<std::string>> alloc_ids;  // per allocation: every id of its container
  size_t unknown = 0;
  if (!cfg_.device_checkpoint.empty()) {
    std::vector<CheckpointEntry> entries;
    std::string cerr;
    ckpt_ok = device_checkpoint_read(cfg_.device_checkpoint, &entries, &cerr);
    if (!ckpt_ok) GPUMON_LOG(LogLevel::kWarn, "kubelet-files", "device checkpoint: " + cerr);
    std::vector<DeviceStatic> st;
    {
      std::lock_guard<std::mutex> g(state_mu_);
      st = *statics_;
    }
    // every container id the log tree knows per (pod uid, container name): a restarted container
    // leaves the dead instance's log link until garbage collection, next to the live one
    std::unordered_map<std::string, std::vector<const ContainerMeta*>> by_uid_ctr;
    std::unordered_map<std::string, const ContainerMeta*> by_uid;
    for (const auto& m : metas)
      if (!m.pod_uid.empty()) {
        by_uid_ctr[m.pod_uid + "/" + m.container_name].push_back(&m);
        by_uid.emplace(m.pod_uid, &m);
      }
    for (const auto& c : entries) {
      if (!starts_with(c.resource, cfg_.pod_resources_prefix)) continue;
      const auto pod = by_uid.find(c.pod_uid);
      if (pod == by_uid.end()) continue;  // not (or no longer) on this node
      const auto ctr = by_uid_ctr.find(c.pod_uid + "/" + c.container_name);
      std::vector<std::string> ids;
      if (ctr != by_uid_ctr.end())
        for (const ContainerMeta* m : ctr->second)
          if (!m->container_id.empty() && std::find(ids.begin(), ids.end(), m->container_id) == ids.end())
            ids.push_back(m->container_id);
      for (const auto& id : c.device_ids) {
        const int idx = match_device_id(id, st);
        if (idx < 0) {
          unknown++;
          continue;
        }
        Allocation a;
        a.pod_namespace = pod->second->pod_namespace;
        a.pod_name = pod->second->pod_name;
        a.pod_uid = c.pod_uid;
        a.container_name = c.container_name;
        if (!ids.empty()) a.container_id = ids.front();
        a.gpu_index = idx;
        allocs.push_back(std::move(a));
        alloc_ids.push_back(ids);
      }
    }
  }
  size_t exited = 0;
  // one /proc/*/cgroup pass per refresh, only when these allocations are used (publish_allocations:
  // not while PodResources is polled) and some carry a container id to check. An allocation is
  // running when ANY of its container's known ids has a live process, and then carries that id.
  if (cfg_.pod_resources_socket.empty() &&
      std::any_of(allocs.begin(), allocs.end(), [](const Allocation& a) { return !a.container_id.empty(); })) {
    std::unordered_set<std::string> running;
    if (running_container_ids(cfg_.attribution.procfs_root, &running)) {
      std::vector<Allocation> kept;
      for (size_t i = 0; i < allocs.size(); ++i) {
        Allocation& a = allocs[i];
        if (a.container_id.empty()) {
          kept.push_back(std::move(a));
          continue;
        }
        const auto& ids = alloc_ids[i];
        auto live = std::find_if(ids.begin(), ids.end(), [&](const std::string& id) { return running.count(id) > 0; });
        if (live == ids.end()) {
          exited++;
          continue;
        }
        a.container_id = *live;
        kept.push_back(std::move(a));
      }
      allocs.swap(kept);
    }
  }
  const size_t n_metas = metas.size();
  {
    std::lock_guard<std::mutex> g(meta_mu_);
    if (logs_ok || cfg_.pod_log_root.empty()) files_metas_ = std::move(metas);
    if (ckpt_ok || cfg_.device_checkpoint.empty()) files_allocs_ = std::move(allocs);
  }
  publish_container_meta();
  publish_allocations();
  std::vector<ExtraSeries> ex;
  if (!cfg_.pod_log_root.empty()) {
    ex.push_back({"gpumon_kubelet_files_up",
                  "1 if the last read of a kubelet-written metadata file succeeded (pod_logs: the /var/log "
                  "containers/ + pods/ trees; device_checkpoint: the device-plugin checkpoint).",
                  "gauge", -1, {{"source", "pod_logs"}}, logs_ok ? 1.0 : 0.0});
    ex.push_back({"gpumon_kubelet_files_containers", "Containers named by the kubelet's log tree.", "gauge", -1, {},
                  static_cast<double>(n_metas)});
  }
  if (!cfg_.device_checkpoint.empty()) {
    ex.push_back({"gpumon_kubelet_files_up",
                  "1 if the last read of a kubelet-written metadata file succeeded (pod_logs: the /var/log "
                  "containers/ + pods/ trees; device_checkpoint: the device-plugin checkpoint).",
                  "gauge", -1, {{"source", "device_checkpoint"}}, ckpt_ok ? 1.0 : 0.0});
    ex.push_back({"gpumon_kubelet_files_unknown_devices", "Checkpointed device IDs that match no local GPU.", "gauge",
                  -1, {}, static_cast<double>(unknown)});
    ex.push_back({"gpumon_kubelet_files_exited_allocations",
                  "Checkpointed GPU allocations left out because their container has no live process (a finished "
                  "pod the kubelet has not deleted yet).",
                  "gauge", -1, {}, static_cast<double>(exited)});
  }
  set_extra("kubelet_files", std::move(ex));
  return logs_ok || ckpt_ok;
}

void Exporter::publish_allocations() {
  std::vector<Allocation> all;
  {
    std::lock_guard<std::mutex> g(meta_mu_);
    all = podres_allocs_;
    all.insert(all.end(), docker_allocs_.begin(), docker_allocs_.end());
    // the device checkpoint says what the kubelet's PodResources says: only when that is not polled
    if (cfg_.pod_resources_socket.empty()) all.insert(all.end(), files_allocs_.begin(), files_allocs_.end());
  }
  attr_->set_allocations(std::move(all));  // a (pod, container, GPU) listed by both is one idle row
}

std::vector<int> Exporter::docker_container_gpus(const DockerInspect& in, const std::vector<DeviceStatic>& st) {
  std::vector<int> out;
  auto add = [&](int i) {
    if (i >= 0 && i < static_cast<int>(st.size()) && std::find(out.begin(), out.end(), i) == out.end())
      out.push_back(i);
  };
  auto all = [&] {
    for (int i = 0; i < static_cast<int>(st.size()); ++i) add(i);
  };
  for (const auto& path : in.devices) {
    std::string p = path;
    while (p.size() > 1 && p.back() == '/') p.pop_back();
    if (p == "/dev/dri") {
      all();
    } else if (starts_with(p, "/dev/dri/renderD") || starts_with(p, "/dev/dri/card")) {
      const bool render = starts_with(p, "/dev/dri/renderD");
      const std::string num = p.substr(render ? 16 : 13);
      if (num.empty() || num.find_first_not_of("0123456789") != std::string::npos) continue;
      const int n = atoi(num.c_str());
      for (size_t i = 0; i < st.size(); ++i)
        if ((render ? st[i].drm_render : st[i].drm_card) == n) add(static_cast<int>(i));
    }
  }
  for (const auto& kv : in.env) {
    if (!starts_with(kv, "AMD_VISIBLE_DEVICES=")) continue;
    const std::string v = kv.substr(20);
    if (v == "all") {
      all();
      continue;
    }
    for (size_t p = 0; p <= v.size();) {
      size_t e = v.find(',', p);
      if (e == std::string::npos) e = v.size();
      const std::string tok = v.substr(p, e - p);
      if (!tok.empty() && tok.find_first_not_of("0123456789") == std::string::npos) add(atoi(tok.c_str()));
      else if (!tok.empty()) add(match_device_id(tok, st));
      p = e + 1;
    }
  }
  std::sort(out.begin(), out.end());
  return out;
}

}  // namespace gpumon
