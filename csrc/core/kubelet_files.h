// Pod metadata and GPU allocations from files the kubelet writes on the node -- the socket-free
// source for an exporter that runs as non-root, where the kubelet PodResources socket (root, 0755)
// and the CRI runtime socket (root, 0660) cannot be connected to (least privilege):
//
//   <log_root>/containers/<pod>_<namespace>_<container>-<container id>.log
//        symlinks the kubelet keeps for log collectors: container id -> pod, namespace, container
//   <log_root>/pods/<namespace>_<pod>_<pod uid>/
//        one directory per pod on the node: pod uid <-> (namespace, pod)
//   /var/lib/kubelet/device-plugins/kubelet_internal_checkpoint
//        the device manager's checkpoint (JSON): pod uid, container, resource, device ids
//        (root 0600 on a default kubelet: readable by a root exporter without any capability, not
//        by a non-root one -- a non-root exporter has no idle-allocation rows)
//
// Pod and namespace names are DNS labels/subdomains and container names DNS labels, so '_' only
// appears as the kubelet's separator. Pod labels are not in these files: the opt-in label gate and
// user_label need the CRI source; the reference's user-name rule works on the pod name alone
// (/root/reference/gpu.py:196-199). Reference counterpart: `docker ps` / `docker inspect` over the
// root-equivalent docker.sock (gpu.py:86-103, gpu_monitor.yaml:24-28).
#pragma once

#include <map>
#include <string>
#include <unordered_set>
#include <utility>
#include <vector>

#include "attribution.h"

namespace gpumon {

// Containers named by <log_root>/containers (+ pod uids from <log_root>/pods). False with *err
// when neither directory can be listed.
bool kubelet_log_metadata(const std::string& log_root, std::vector<ContainerMeta>* out, std::string* err);

// "<pod>_<namespace>_<container>-<64 hex id>.log" -> parts; false for any other name.
bool parse_container_log_name(const std::string& name, std::string* pod, std::string* ns, std::string* container,
                              std::string* id);
// "<namespace>_<pod>_<uid>" -> parts.
bool parse_pod_log_dir(const std::string& name, std::string* ns, std::string* pod, std::string* uid);

struct CheckpointEntry {
  std::string pod_uid, container_name, resource;
  std::vector<std::string> device_ids;
};

// Body of kubelet_internal_checkpoint: {"Data": {"PodDeviceEntries": [{"PodUID", "ContainerName",
// "ResourceName", "DeviceIDs": {"<numa>": [ids]} (v2) or [ids] (v1), "AllocResp"}], ...}, "Checksum"}.
bool device_checkpoint_parse(const std::string& json, std::vector<CheckpointEntry>* out, std::string* err);
bool device_checkpoint_read(const std::string& path, std::vector<CheckpointEntry>* out, std::string* err);

// Container ids that have at least one live process: /proc/<pid>/cgroup of every process
// (parse_cgroup). The checkpoint keeps entries of pods that finished but were not deleted (the
// kubelet prunes them at its next Allocate), and their containers have no process left. False when
// the scan cannot tell: procfs unreadable, or no container other than the reader's own is visible
// (not in the host PID namespace).
bool running_container_ids(const std::string& procfs_root, std::unordered_set<std::string>* out);

}  // namespace gpumon
