// Kubelet-written files as a pod metadata / allocation source (kubelet_files.h).
#include "kubelet_files.h"

#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <unordered_map>

#include "common.h"
#include "json_lite.h"

namespace gpumon {

namespace {

bool hex64(const std::string& s) {
  if (s.size() != 64) return false;
  for (char c : s)
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
  return true;
}

bool list_dir(const std::string& dir, std::vector<std::string>* names, std::string* err) {
  names->clear();
  DIR* d = opendir(dir.c_str());
  if (!d) {
    if (err) *err = dir + ": " + strerror(errno);
    return false;
  }
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    names->emplace_back(e->d_name);
  }
  closedir(d);
  return true;
}

constexpr size_t kMaxCheckpoint = 16u << 20;

}  // namespace

bool parse_container_log_name(const std::string& name, std::string* pod, std::string* ns, std::string* container,
                              std::string* id) {
  if (!ends_with(name, ".log")) return false;
  const std::string stem = name.substr(0, name.size() - 4);
  const size_t a = stem.find('_');
  if (a == std::string::npos || a == 0) return false;
  const size_t b = stem.find('_', a + 1);
  if (b == std::string::npos || b == a + 1 || stem.find('_', b + 1) != std::string::npos) return false;
  const std::string rest = stem.substr(b + 1);  // <container>-<id>
  const size_t dash = rest.rfind('-');
  if (dash == std::string::npos || dash == 0) return false;
  const std::string cid = rest.substr(dash + 1);
  if (!hex64(cid)) return false;
  *pod = stem.substr(0, a);
  *ns = stem.substr(a + 1, b - a - 1);
  *container = rest.substr(0, dash);
  *id = cid;
  return true;
}

bool parse_pod_log_dir(const std::string& name, std::string* ns, std::string* pod, std::string* uid) {
  const size_t a = name.find('_');
  const size_t b = name.rfind('_');
  if (a == std::string::npos || b == a || a == 0 || b == a + 1 || b + 1 >= name.size()) return false;
  *ns = name.substr(0, a);
  *pod = name.substr(a + 1, b - a - 1);
  *uid = name.substr(b + 1);
  return pod->find('_') == std::string::npos;
}

bool running_container_ids(const std::string& procfs_root, std::unordered_set<std::string>* out) {
  out->clear();
  DIR* d = opendir(procfs_root.c_str());
  if (!d) return false;
  std::string text, self;
  if (read_file(procfs_root + "/self/cgroup", &text, 65536)) self = parse_cgroup(text).container_id;
  while (struct dirent* ent = readdir(d)) {
    const char* n = ent->d_name;
    if (*n < '1' || *n > '9') continue;  // pids only
    if (!read_file(procfs_root + "/" + n + "/cgroup", &text, 65536)) continue;  // exited meanwhile
    CgroupInfo cg = parse_cgroup(text);
    if (cg.found) out->insert(std::move(cg.container_id));
  }
  closedir(d);
  for (const auto& id : *out)
    if (id != self) return true;
  return false;
}

bool kubelet_log_metadata(const std::string& log_root, std::vector<ContainerMeta>* out, std::string* err) {
  out->clear();
  std::vector<std::string> pods, ctrs;
  std::string e1, e2;
  const bool have_pods = list_dir(log_root + "/pods", &pods, &e1);
  const bool have_ctrs = list_dir(log_root + "/containers", &ctrs, &e2);
  if (!have_pods && !have_ctrs) {
    if (err) *err = e1 + "; " + e2;
    return false;
  }
  std::unordered_map<std::string, std::string> uid_of;  // "ns/pod" -> uid
  for (const auto& d : pods) {
    std::string ns, pod, uid;
    if (parse_pod_log_dir(d, &ns, &pod, &uid)) uid_of[ns + "/" + pod] = uid;
  }
  for (const auto& f : ctrs) {
    ContainerMeta m;
    if (!parse_container_log_name(f, &m.pod_name, &m.pod_namespace, &m.container_name, &m.container_id)) continue;
    const auto it = uid_of.find(m.pod_namespace + "/" + m.pod_name);
    if (it != uid_of.end()) m.pod_uid = it->second;
    out->push_back(std::move(m));
  }
  return true;
}

bool device_checkpoint_parse(const std::string& json, std::vector<CheckpointEntry>* out, std::string* err) {
  out->clear();
  JsonReader r(json);
  auto entry = [&]() {
    CheckpointEntry c;
    const bool ok = r.members([&](const std::string& k) {
      if (k == "PodUID" && r.peek('"')) return r.string(&c.pod_uid);
      if (k == "ContainerName" && r.peek('"')) return r.string(&c.container_name);
      if (k == "ResourceName" && r.peek('"')) return r.string(&c.resource);
      if (k == "DeviceIDs") {
        if (r.peek('[')) {  // checkpoint v1: a plain list
          std::vector<std::string> ids;
          if (!r.string_array(&ids)) return false;
          c.device_ids.insert(c.device_ids.end(), ids.begin(), ids.end());
          return true;
        }
        return r.members([&](const std::string&) {  // v2: NUMA node -> list
          std::vector<std::string> ids;
          if (!r.string_array(&ids)) return false;
          c.device_ids.insert(c.device_ids.end(), ids.begin(), ids.end());
          return true;
        });
      }
      return r.skip(3);
    });
    if (ok && !c.pod_uid.empty()) out->push_back(std::move(c));
    return ok;
  };
  const bool ok = r.members([&](const std::string& k) {
    if (k != "Data") return r.skip(1);
    return r.members([&](const std::string& dk) { return dk == "PodDeviceEntries" ? r.elements(entry) : r.skip(2); });
  });
  if (!ok || !r.at_end()) {
    if (err) *err = r.ok() ? "malformed device-plugin checkpoint" : r.error();
    out->clear();
    return false;
  }
  return true;
}

bool device_checkpoint_read(const std::string& path, std::vector<CheckpointEntry>* out, std::string* err) {
  const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    if (err) *err = path + ": " + strerror(errno);
    return false;
  }
  std::string body;
  char buf[65536];
  for (;;) {
    const ssize_t n = ::read(fd, buf, sizeof buf);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) break;
    body.append(buf, static_cast<size_t>(n));
    if (body.size() > kMaxCheckpoint) {
      ::close(fd);
      if (err) *err = path + ": larger than 16 MiB";
      return false;
    }
  }
  ::close(fd);
  return device_checkpoint_parse(body, out, err);
}

}  // namespace gpumon
