// PID -> container -> pod attribution, user-name derivation and the opt-in gate.
//
// Reference parity (/root/reference/gpu.py):
//   - gpu.py:174-178  `docker top <cid> -eo pid` per container, then keep GPU processes whose pid
//                     is in that list                    -> here: /proc/<pid>/cgroup, one read per
//                     new pid, cached by (pid, starttime) (fixes the pid-reuse race).
//   - gpu.py:184-189  opt-in gate: docker label mlgpu == "mlgpu"       -> OptIn (configurable
//                     key=value over container AND pod labels, fixes Q13; empty = everyone).
//   - gpu.py:193-199  pod name / namespace from io.kubernetes.* docker labels, user_name from the
//                     pod name (turing-gpu-notebook-<user>-x-y or <a>-<user>-...)
//                                                        -> derive_user(): same rule, but a pod
//                     name without '-' yields "-" instead of crashing (Q2); a regex or a pod label
//                     may override.
// Container/pod metadata (the docker-inspect equivalent) is pushed in by the control plane
// (tests/oracles/attribution, the Python oracle: CRI ListContainers / ListPodSandbox, kubelet PodResources). When no table
// entry exists, an optional procfs fallback reads HOSTNAME and the service-account namespace of
// the process itself.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <regex>
#include <string>
#include <unordered_map>
#include <vector>

namespace gpumon {

struct CgroupInfo {
  bool found = false;         // a container id was recognised
  std::string runtime;        // docker | containerd | crio | unknown
  std::string container_id;   // full (usually 64 hex) id
  std::string pod_uid;        // with dashes, if the path carries one
  std::string qos;            // guaranteed | burstable | besteffort
};

// Parses the text of /proc/<pid>/cgroup (v1 or v2; cgroupfs or systemd drivers; docker,
// containerd/cri-containerd, cri-o).
CgroupInfo parse_cgroup(const std::string& text);

struct ContainerMeta {
  std::string container_id;     // full runtime id (match key)
  std::string container_name;
  std::string pod_name;
  std::string pod_namespace;
  std::string pod_uid;
  std::string user_name;        // optional override (e.g. from the control plane)
  std::map<std::string, std::string> labels;  // container labels U pod labels U annotations
};

struct Allocation {
  std::string pod_namespace, pod_name, container_name, container_id, pod_uid;
  int gpu_index = -1;           // index into the exporter's device list
  std::map<std::string, std::string> labels;
  std::string user_name;
};

struct AttributionConfig {
  std::string procfs_root = "/proc";
  std::string opt_in = "";                  // "key=value"; empty = no gate (all pods)
  std::string user_label = "";              // pod/container label carrying the user name
  std::string user_regex = "";              // ECMAScript regex on pod name; group 1 = user
  std::string user_prefix = "turing-gpu-notebook-";  // reference rule prefix (gpu.py:196)
  bool compat_user_rule = true;
  bool procfs_env_fallback = true;          // HOSTNAME + SA namespace of the process
  bool include_host_processes = true;       // GPU processes not in any container
  // amdsmi reports KFD (host-namespace) PIDs. Without hostPID the same number in our /proc can be
  // an unrelated process: require /proc/<pid>/fd to hold /dev/kfd before trusting /proc/<pid>
  // (an unreadable fd dir is treated as "unknown", not as a mismatch).
  bool verify_kfd = true;
  // Pod / container label keys copied onto the pod_gpu_* series as label_<key> (non [A-Za-z0-9_]
  // characters -> '_'), like kube-state-metrics' --metric-labels-allowlist. Empty = none.
  std::vector<std::string> label_allowlist;
};

using LabelPairs = std::vector<std::pair<std::string, std::string>>;

struct ProcIdentity {
  bool valid = false;           // /proc/<pid> readable
  bool pid_mismatch = false;    // /proc/<pid> exists but does not hold /dev/kfd (other pid ns)
  bool in_container = false;
  bool opted_in = true;
  uint64_t starttime = 0;
  std::string comm;
  std::string runtime;
  std::string container_id;
  std::string container_name;
  std::string pod_name = "-";
  std::string pod_namespace = "-";
  std::string pod_uid;
  std::string user_name = "-";
  std::string source;           // meta | procfs | none
  LabelPairs extra_labels;      // allowlisted pod labels (label_<key>, value)
};

class Attributor {
 public:
  explicit Attributor(AttributionConfig cfg);

  void set_container_meta(std::vector<ContainerMeta> metas);
  void set_allocations(std::vector<Allocation> allocs);
  std::vector<Allocation> allocations() const;
  size_t meta_size() const;

  ProcIdentity resolve(uint32_t pid);
  // Drops cache entries for pids not in `alive` (call once per tick with the live pid set).
  void gc(const std::vector<uint32_t>& alive);

  std::string derive_user(const std::string& pod_name,
                          const std::map<std::string, std::string>& labels) const;
  bool opted_in(const std::map<std::string, std::string>& labels) const;
  // Allowlisted labels present in `labels`, as (prometheus label name, value) in allowlist order.
  LabelPairs export_labels(const std::map<std::string, std::string>& labels) const;
  const AttributionConfig& config() const { return cfg_; }

  uint64_t cache_hits() const { return hits_; }
  uint64_t cache_misses() const { return misses_; }

 private:
  struct CacheEntry {
    uint64_t starttime = 0;
    CgroupInfo cg;
    std::string comm;
    std::string env_pod, env_ns;  // procfs fallback values
    bool env_done = false;
    int kfd = -1;                 // 1 holds /dev/kfd, 0 does not, -1 unknown (unreadable)
  };
  int holds_kfd(uint32_t pid) const;
  AttributionConfig cfg_;
  std::unique_ptr<std::regex> user_re_;
  std::string opt_key_, opt_val_;
  std::vector<std::pair<std::string, std::string>> allow_;  // (label key, prometheus name)
  mutable std::mutex mu_;
  std::shared_ptr<const std::unordered_map<std::string, ContainerMeta>> by_cid_;
  std::shared_ptr<const std::unordered_map<std::string, ContainerMeta>> by_pod_uid_;
  std::vector<Allocation> allocs_;
  std::unordered_map<uint32_t, CacheEntry> cache_;
  uint64_t hits_ = 0, misses_ = 0;

  bool read_stat(uint32_t pid, uint64_t* starttime, std::string* comm) const;
  bool task_stat_ = false;  // read the leader thread's stat (procfs_root has task/ dirs)
  void read_env_fallback(uint32_t pid, CacheEntry* e) const;
};

// Reference rule, exactly (gpu.py:196-199), with the Q2 crash turned into "-".
std::string compat_user_from_pod(const std::string& pod_name, const std::string& prefix);

}  // namespace gpumon
