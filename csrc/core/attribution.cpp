#include "attribution.h"

#include <dirent.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstring>
#include <unordered_set>

#include "common.h"

namespace gpumon {

static bool is_hex_id(std::string_view s) {
  if (s.size() < 32 || s.size() > 128) return false;
  for (char c : s)
    if (!std::isxdigit(static_cast<unsigned char>(c))) return false;
  return true;
}

// Returns true and fills runtime/id if `seg` is a container scope/segment.
static bool match_container_segment(std::string_view seg, std::string_view prev, CgroupInfo* out) {
  struct Pfx {
    const char* prefix;
    const char* runtime;
  };
  static const Pfx kPfx[] = {{"cri-containerd-", "containerd"}, {"docker-", "docker"},
                             {"crio-", "crio"},                 {"libpod-", "podman"},
                             {"containerd-", "containerd"}};
  std::string_view s = seg;
  if (ends_with(s, ".scope")) s.remove_suffix(6);
  for (const auto& p : kPfx) {
    if (starts_with(s, p.prefix)) {
      std::string_view id = s.substr(strlen(p.prefix));
      if (starts_with(id, "conmon-")) return false;  // cri-o monitor, not the workload
      if (is_hex_id(id)) {
        out->runtime = p.runtime;
        out->container_id = std::string(id);
        return true;
      }
    }
  }
  if (is_hex_id(s)) {
    out->runtime = prev == "docker" ? "docker" : (prev.empty() ? "unknown" : "cgroupfs");
    out->container_id = std::string(s);
    return true;
  }
  return false;
}

static void match_pod_segment(std::string_view seg, CgroupInfo* out) {
  // cgroupfs:  pod<uid-with-dashes>
  // systemd:   kubepods-<qos>-pod<uid_with_underscores>.slice / kubepods-pod<uid>.slice
  std::string_view s = seg;
  if (ends_with(s, ".slice")) s.remove_suffix(6);
  size_t p = s.rfind("pod");
  if (p == std::string_view::npos) return;
  if (p != 0 && s[p - 1] != '-') return;
  std::string uid(s.substr(p + 3));
  if (uid.size() < 32) return;
  std::replace(uid.begin(), uid.end(), '_', '-');
  for (char c : uid)
    if (!(std::isxdigit(static_cast<unsigned char>(c)) || c == '-')) return;
  out->pod_uid = uid;
}

static void match_qos(std::string_view seg, CgroupInfo* out) {
  if (seg.find("besteffort") != std::string_view::npos) out->qos = "besteffort";
  else if (seg.find("burstable") != std::string_view::npos) out->qos = "burstable";
}

CgroupInfo parse_cgroup(const std::string& text) {
  CgroupInfo best;
  for (const auto& line_s : split(text, '\n')) {
    std::string_view line = trim(line_s);
    if (line.empty()) continue;
    // hierarchy-id:controllers:path ; the path itself may contain ':'
    size_t c1 = line.find(':');
    if (c1 == std::string_view::npos) continue;
    size_t c2 = line.find(':', c1 + 1);
    if (c2 == std::string_view::npos) continue;
    std::string_view path = line.substr(c2 + 1);
    CgroupInfo cur;
    std::string_view prev;
    bool kube = path.find("kubepods") != std::string_view::npos;
    for (const auto& seg_s : split(path, '/')) {
      std::string_view seg = seg_s;
      if (seg.empty()) continue;
      if (kube) {
        match_pod_segment(seg, &cur);
        match_qos(seg, &cur);
      }
      CgroupInfo tmp;
      if (match_container_segment(seg, prev, &tmp)) {
        cur.found = true;
        cur.runtime = tmp.runtime;
        cur.container_id = tmp.container_id;
      }
      prev = seg;
    }
    if (kube && cur.found && cur.qos.empty()) cur.qos = "guaranteed";
    if (cur.found) {
      if (!best.found || (best.pod_uid.empty() && !cur.pod_uid.empty())) best = cur;
    } else if (!best.found && !cur.pod_uid.empty() && best.pod_uid.empty()) {
      best.pod_uid = cur.pod_uid;
      best.qos = cur.qos;
    }
  }
  return best;
}

std::string compat_user_from_pod(const std::string& pod, const std::string& prefix) {
  if (pod.empty() || pod == "-") return "-";
  if (!prefix.empty()) {
    size_t p = pod.find(prefix);
    if (p != std::string::npos) {
      // Python: pod.split(prefix)[1] -> text between the 1st and 2nd occurrence of prefix
      size_t b = p + prefix.size();
      size_t e = pod.find(prefix, b);
      std::string tail = pod.substr(b, e == std::string::npos ? std::string::npos : e - b);
      // .rsplit("-", 2)[0]
      std::string s = tail;
      for (int k = 0; k < 2; ++k) {
        size_t d = s.rfind('-');
        if (d == std::string::npos) break;
        s.resize(d);
      }
      return s.empty() ? "-" : s;
    }
  }
  // Python: pod.split("-")[1]; IndexError (agent crash, Q2) -> "-"
  size_t d = pod.find('-');
  if (d == std::string::npos) return "-";
  size_t e = pod.find('-', d + 1);
  std::string s = pod.substr(d + 1, e == std::string::npos ? std::string::npos : e - d - 1);
  return s.empty() ? "-" : s;
}

Attributor::Attributor(AttributionConfig cfg) : cfg_(std::move(cfg)) {
  // A real procfs has per-thread directories: the leader thread's stat (task/<pid>/stat) carries
  // the same comm and starttime as the process's, without summing the CPU times of every thread
  // (a PyTorch tenant runs dozens; ~8 vs ~3.5 us per read with 200 threads). A fake tree in the
  // tests has <pid>/stat only.
  task_stat_ = access((cfg_.procfs_root + "/self/task").c_str(), R_OK) == 0;
  if (!cfg_.user_regex.empty()) {
    try {
      user_re_ = std::make_unique<std::regex>(cfg_.user_regex, std::regex::ECMAScript);
    } catch (const std::regex_error& e) {
      GPUMON_LOG(LogLevel::kWarn, "attribution", "invalid --user-regex ignored: " + cfg_.user_regex);
    }
  }
  if (!cfg_.opt_in.empty()) {
    size_t eq = cfg_.opt_in.find('=');
    opt_key_ = cfg_.opt_in.substr(0, eq);
    opt_val_ = eq == std::string::npos ? "" : cfg_.opt_in.substr(eq + 1);
  }
  for (const auto& key : cfg_.label_allowlist) {
    if (key.empty()) continue;
    std::string name = "label_";
    for (char c : key)
      name.push_back((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') ? c : '_');
    bool dup = false;
    for (const auto& kv : allow_) dup = dup || kv.second == name;
    if (dup) {  // "app.kubernetes.io/name" and "app_kubernetes_io_name" would collide: first one wins
      GPUMON_LOG(LogLevel::kWarn, "attribution", "label allowlist: " + key + " collides with an earlier key");
      continue;
    }
    allow_.emplace_back(key, name);
  }
  by_cid_ = std::make_shared<std::unordered_map<std::string, ContainerMeta>>();
  by_pod_uid_ = std::make_shared<std::unordered_map<std::string, ContainerMeta>>();
}

void Attributor::set_container_meta(std::vector<ContainerMeta> metas) {
  auto cid = std::make_shared<std::unordered_map<std::string, ContainerMeta>>();
  auto pod = std::make_shared<std::unordered_map<std::string, ContainerMeta>>();
  for (auto& m : metas) {
    if (!m.pod_uid.empty() && !pod->count(m.pod_uid)) {
      ContainerMeta pm = m;
      pm.container_id.clear();
      pm.container_name.clear();
      (*pod)[m.pod_uid] = std::move(pm);
    }
    if (!m.container_id.empty()) {
      std::string key = m.container_id;
      (*cid)[key] = std::move(m);
    }
  }
  std::lock_guard<std::mutex> g(mu_);
  by_cid_ = std::move(cid);
  by_pod_uid_ = std::move(pod);
}

void Attributor::set_allocations(std::vector<Allocation> allocs) {
  std::lock_guard<std::mutex> g(mu_);
  allocs_ = std::move(allocs);
}

std::vector<Allocation> Attributor::allocations() const {
  std::lock_guard<std::mutex> g(mu_);
  return allocs_;
}

size_t Attributor::meta_size() const {
  std::lock_guard<std::mutex> g(mu_);
  return by_cid_->size();
}

bool Attributor::read_stat(uint32_t pid, uint64_t* starttime, std::string* comm) const {
  std::string s;
  const std::string ps = std::to_string(pid);
  if (!read_file(cfg_.procfs_root + "/" + ps + (task_stat_ ? "/task/" + ps + "/stat" : "/stat"), &s, 4096)) return false;
  // pid (comm) state ppid ... ; comm may contain spaces/parens: use the LAST ')'
  size_t lp = s.find('('), rp = s.rfind(')');
  if (lp == std::string::npos || rp == std::string::npos || rp < lp) return false;
  *comm = s.substr(lp + 1, rp - lp - 1);
  // fields after ") ": state(3) ppid(4) ... starttime is field 22 -> index 19 after state. Walked
  // in place (every process, every tick): no vector of 50 field strings.
  size_t p = rp + 2;
  for (int k = 0; k < 19 && p < s.size(); ++k) {
    p = s.find(' ', p);
    if (p == std::string::npos) break;
    ++p;
  }
  *starttime = p != std::string::npos && p < s.size() ? strtoull(s.c_str() + p, nullptr, 10) : 0;
  return true;
}

int Attributor::holds_kfd(uint32_t pid) const {
  std::string dir = cfg_.procfs_root + "/" + std::to_string(pid) + "/fd";
  DIR* d = opendir(dir.c_str());
  if (!d) return -1;
  int found = 0;
  char link[256];
  int scanned = 0;
  while (struct dirent* ent = readdir(d)) {
    if (ent->d_name[0] == '.') continue;
    if (++scanned > 65536) break;
    ssize_t n = readlink((dir + "/" + ent->d_name).c_str(), link, sizeof link - 1);
    if (n <= 0) continue;
    link[n] = 0;
    if (strcmp(link, "/dev/kfd") == 0) {
      found = 1;
      break;
    }
  }
  closedir(d);
  return found;
}

void Attributor::read_env_fallback(uint32_t pid, CacheEntry* e) const {
  e->env_done = true;
  std::string base = cfg_.procfs_root + "/" + std::to_string(pid);
  std::string env;
  if (read_file(base + "/environ", &env, 1 << 20)) {
    size_t pos = 0;
    while (pos < env.size()) {
      size_t end = env.find('\0', pos);
      if (end == std::string::npos) end = env.size();
      std::string_view kv(env.data() + pos, end - pos);
      if (starts_with(kv, "HOSTNAME=")) e->env_pod = std::string(kv.substr(9));
      if (starts_with(kv, "POD_NAME=")) e->env_pod = std::string(kv.substr(9));
      if (starts_with(kv, "POD_NAMESPACE=")) e->env_ns = std::string(kv.substr(14));
      pos = end + 1;
    }
  }
  if (e->env_ns.empty()) {
    std::string ns;
    if (read_file(base + "/root/var/run/secrets/kubernetes.io/serviceaccount/namespace", &ns, 256))
      e->env_ns = std::string(trim(ns));
  }
}

ProcIdentity Attributor::resolve(uint32_t pid) {
  ProcIdentity id;
  uint64_t st = 0;
  std::string comm;
  if (!read_stat(pid, &st, &comm)) return id;  // not visible (other pid namespace, exited)
  id.valid = true;
  id.starttime = st;
  id.comm = comm;
  std::shared_ptr<const std::unordered_map<std::string, ContainerMeta>> by_cid, by_pod;
  CacheEntry* e = nullptr;
  {
    std::lock_guard<std::mutex> g(mu_);
    by_cid = by_cid_;
    by_pod = by_pod_uid_;
    auto it = cache_.find(pid);
    if (it != cache_.end() && it->second.starttime == st) {
      ++hits_;
      e = &it->second;
    } else {
      ++misses_;
      CacheEntry ne;
      ne.starttime = st;
      ne.comm = comm;
      if (cfg_.verify_kfd) ne.kfd = holds_kfd(pid);
      std::string cg;
      if (ne.kfd != 0 &&
          read_file(cfg_.procfs_root + "/" + std::to_string(pid) + "/cgroup", &cg, 65536))
        ne.cg = parse_cgroup(cg);
      cache_[pid] = std::move(ne);
      e = &cache_[pid];
    }
  }
  // `e` stays valid: only this (sampler) thread inserts/erases cache entries.
  if (e->kfd == 0) {
    // Same number, different process (exporter not in the host PID namespace): attribute nothing.
    id.valid = false;
    id.pid_mismatch = true;
    id.comm.clear();
    id.source = "pidns";
    id.opted_in = opted_in({}) && cfg_.include_host_processes;
    return id;
  }
  const CgroupInfo& cg = e->cg;
  id.in_container = cg.found;
  id.runtime = cg.runtime;
  id.container_id = cg.container_id;
  id.pod_uid = cg.pod_uid;
  const ContainerMeta* m = nullptr;
  if (cg.found) {
    auto it = by_cid->find(cg.container_id);
    if (it != by_cid->end()) m = &it->second;
  }
  if (!m && !cg.pod_uid.empty()) {
    auto it = by_pod->find(cg.pod_uid);
    if (it != by_pod->end()) m = &it->second;
  }
  std::map<std::string, std::string> empty;
  const std::map<std::string, std::string>* labels = &empty;
  if (m) {
    id.source = "meta";
    id.pod_name = m->pod_name.empty() ? "-" : m->pod_name;
    id.pod_namespace = m->pod_namespace.empty() ? "-" : m->pod_namespace;
    id.container_name = m->container_name;
    labels = &m->labels;
    id.user_name = !m->user_name.empty() ? m->user_name : derive_user(id.pod_name, m->labels);
    id.extra_labels = export_labels(m->labels);
  } else if (cg.found && cfg_.procfs_env_fallback) {
    if (!e->env_done) read_env_fallback(pid, e);
    if (!e->env_pod.empty()) {
      id.source = "procfs";
      id.pod_name = e->env_pod;
      id.pod_namespace = e->env_ns.empty() ? "-" : e->env_ns;
      id.user_name = derive_user(id.pod_name, empty);
    } else {
      id.source = "none";
    }
  } else {
    id.source = "none";
  }
  id.opted_in = opted_in(*labels);
  if (!cg.found && !cfg_.include_host_processes) id.opted_in = false;
  return id;
}

LabelPairs Attributor::export_labels(const std::map<std::string, std::string>& labels) const {
  LabelPairs out;
  for (const auto& [key, name] : allow_) {
    auto it = labels.find(key);
    if (it != labels.end() && !it->second.empty()) out.emplace_back(name, it->second);
  }
  return out;
}

void Attributor::gc(const std::vector<uint32_t>& alive) {
  std::unordered_set<uint32_t> keep(alive.begin(), alive.end());
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = cache_.begin(); it != cache_.end();) {
    if (!keep.count(it->first)) it = cache_.erase(it);
    else ++it;
  }
}

std::string Attributor::derive_user(const std::string& pod_name,
                                    const std::map<std::string, std::string>& labels) const {
  if (!cfg_.user_label.empty()) {
    auto it = labels.find(cfg_.user_label);
    if (it != labels.end() && !it->second.empty()) return it->second;
  }
  if (user_re_) {
    std::smatch mm;
    if (std::regex_search(pod_name, mm, *user_re_) && mm.size() > 1 && mm[1].length() > 0)
      return mm[1].str();
  }
  if (cfg_.compat_user_rule) return compat_user_from_pod(pod_name, cfg_.user_prefix);
  return "-";
}

bool Attributor::opted_in(const std::map<std::string, std::string>& labels) const {
  if (opt_key_.empty()) return true;
  auto it = labels.find(opt_key_);
  return it != labels.end() && it->second == opt_val_;
}

}  // namespace gpumon
