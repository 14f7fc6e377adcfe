// Configuration of the standalone exporter binary: the same keys, file format and precedence as the
// Python control plane (gpumon/config.py), so one ConfigMap (deploy/k8s/gpumon-daemonset.yaml)
// drives either `python -m gpumon serve --config` or `bin/gpumon-exporter --config`.
//
//   defaults < YAML file (--config PATH or GPUMON_CONFIG) < environment < command-line flags
//
// Environment: the reference's NODE_NAME and INFLUXDB_URL (/root/reference/gpu.py:19-20) plus
// GPUMON_<KEY> for every key. The file format is the YAML subset the ConfigMap uses: an optional
// top-level `gpumon:` mapping, `key: value` scalars (plain / single / double quoted), flow lists
// `[a, b]` and block lists (`- a`), `#` comments. No anchors, no multi-line scalars, no nesting
// below the one mapping level — a file needing more is a configuration error, reported with its line.
#pragma once

#include <map>
#include <string>
#include <vector>

#include "exporter.h"
#include "ondevice.h"

namespace gpumon {

struct NativeOptions {
  ExporterConfig cfg;
  OnDeviceConfig od;
  std::string listen = ":9400";          // every address, dual-stack where the kernel has IPv6
  std::string pod_resources_socket = "/var/lib/kubelet/pod-resources/kubelet.sock";  // "" = off
  std::string cri_socket;                 // "" = autodetect, "none" = off
  int probe_every = 1;                    // probe period in sampler intervals
  double metadata_refresh_s = 10.0;
  std::vector<std::string> resource_names = {"amd.com/gpu"};
  std::string log_level = "info";
};

// key -> list of values (a scalar is a one-element list). Keys keep file order in `order`.
struct YamlDoc {
  std::map<std::string, std::vector<std::string>> values;
  std::vector<std::string> order;
};

// Parses the YAML subset described above; false with "line N: ..." in err.
bool parse_yaml_subset(const std::string& text, YamlDoc* doc, std::string* err);

// Sets one key (Python Config field name). Returns 1 = applied, 0 = unknown key (Python-only keys
// such as control_plane land here), -1 = bad value (err set).
int options_set(NativeOptions* o, const std::string& key, const std::vector<std::string>& vals, std::string* err);

// YAML file: unknown keys are returned in `unknown` (warned about, not fatal); bad values fail.
bool options_load_file(NativeOptions* o, const std::string& path, std::vector<std::string>* unknown, std::string* err);

// NODE_NAME, INFLUXDB_URL, GPUMON_<KEY> (GPUMON_CONFIG / GPUMON_AMDSMI_LIB excluded, as in Python).
bool options_apply_env(NativeOptions* o, char** envp, std::string* err);

// Resolves listen address, sockets and the on-device cadence into cfg / od (after all sources).
// false with *err for a listen address parse_listen refuses.
bool options_finalize(NativeOptions* o, std::string* err);

// Effective configuration as one JSON object (Python field names), for --print-config.
std::string options_json(const NativeOptions& o);

}  // namespace gpumon
