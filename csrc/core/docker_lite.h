// Read-only Docker Engine API client for plain-Docker GPU nodes (no CRI runtime in front of the
// containers): GET /containers/json over the daemon's unix socket, HTTP/1.0, parsed with a small
// bounded JSON reader. Container labels (io.kubernetes.pod.name / .namespace / .container.name on
// dockershim-era kubelets, arbitrary user labels such as the reference's `mlgpu` opt-in label)
// become ContainerMeta the same way the CRI poller's do.
//
// Reference parity: the reference shells out to `docker inspect <id>` once per GPU container per
// cycle and json-decodes the labels (/root/reference/gpu.py:86-88,184-195), plus `docker ps` /
// `docker top` (gpu.py:92-103,177). Here one listing per metadata refresh serves every container,
// off the sampling tick, and the process -> container mapping stays on /proc/<pid>/cgroup.
// The docker socket is root-equivalent: this client only sends GETs (the listing, and one inspect
// per new container for its GPU devices), and the exporter uses it only when `docker_socket` is
// configured (never autodetected).
#pragma once

#include <map>
#include <string>
#include <vector>

namespace gpumon {

struct DockerContainer {
  std::string id;      // full 64-hex id
  std::string name;    // Names[0] without the leading '/'
  std::string state;   // running | paused | ...
  std::map<std::string, std::string> labels;
};

// The parts of GET /containers/{id}/json (docker inspect) that say which GPUs a container holds.
struct DockerInspect {
  std::string id;
  std::vector<std::string> devices;  // HostConfig.Devices[].PathOnHost (/dev/dri/renderD128, /dev/dri, ...)
  std::vector<std::string> env;      // Config.Env ("AMD_VISIBLE_DEVICES=0,1" from the AMD container toolkit)
};

// Parses the JSON body of GET /containers/json. Unknown members are skipped; nesting depth and
// string escapes are bounded/validated. Returns false (with *err) on malformed input.
bool docker_parse_containers(const std::string& json, std::vector<DockerContainer>* out, std::string* err);

// Splits a raw HTTP/1.x response (status line, headers, body delimited by Content-Length,
// chunked transfer coding, or connection close) into status + body. `eof`: the peer has closed
// the connection; without it a close-delimited body is reported incomplete (false).
bool http1_parse_response(const std::string& raw, int* status, std::string* body, std::string* err,
                          bool eof = true);

bool docker_parse_inspect(const std::string& json, DockerInspect* out, std::string* err);

// GET /containers/{id}/json (id: hex only, checked).
bool docker_inspect(const std::string& socket_path, const std::string& id, DockerInspect* out, std::string* err,
                    int timeout_ms = 3000, int* http_status = nullptr);

// GET /containers/json on `socket_path` (optionally "unix://"-prefixed). *http_status receives the
// HTTP status (-1: transport failure).
bool docker_list(const std::string& socket_path, std::vector<DockerContainer>* out, std::string* err,
                 int timeout_ms = 3000, int* http_status = nullptr);

}  // namespace gpumon
