// The exporter's configuration: the ONE implementation of its keys, defaults, value coercion, flag
// vocabulary, precedence and autodetects. bin/gpumon-exporter parses its command line here, and the
// Python side (gpumon/config.py, `gpumon serve`) is a view over the same NativeOptions through the
// bindings, so one ConfigMap (deploy/k8s/gpumon-daemonset.yaml) drives either entry point with no
// second copy to drift. The reference's whole configuration was two env vars
// and constants (/root/reference/gpu.py:17-26).
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
  NativeOptions() { cfg.host.clear(); }  // "" until options_finalize: NODE_NAME > host name > "no_name"
  ExporterConfig cfg;
  OnDeviceConfig od;
  std::string listen = ":9400";          // every address, dual-stack where the kernel has IPv6
  std::string pod_resources_socket = "/var/lib/kubelet/pod-resources/kubelet.sock";  // "" = off
  std::string cri_socket;                 // "" = autodetect (cri_autodetect_sockets), "none" = off
  std::string control_plane = "native";   // native | off (no kubelet / CRI / Docker / log-tree pollers)
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

// One configuration key: name, documentation section and help (docs/configuration.md is generated
// from these through the bindings).
struct OptionKey {
  const char* key;
  const char* section;
  const char* help;
};
const std::vector<OptionKey>& option_keys();

// One command-line flag: it sets `key` to the next argument (or to `fixed` when that is non-null).
// `aliases` is a comma-separated list of other spellings.
struct OptionFlag {
  const char* flag;
  const char* aliases;
  const char* key;
  const char* fixed;
  const char* help;
};
const std::vector<OptionFlag>& option_flags();

// Sets one key. Returns 1 = applied, 0 = unknown key, -1 = bad value (err set).
int options_set(NativeOptions* o, const std::string& key, const std::vector<std::string>& vals, std::string* err);

// The whole precedence over a command line: YAML file (--config PATH, else GPUMON_CONFIG from envp)
// < environment < --compat < flags (option_flags, in order; `--flag=value` too). Arguments that
// are not configuration flags go to `rest` (nullptr: an error). Unknown file keys -> `warnings`.
enum class ParseStatus { kOk = 0, kBadFile, kBadEnv, kBadFlag, kBadValue };
ParseStatus options_parse(NativeOptions* o, const std::vector<std::string>& args, char** envp,
                          std::vector<std::string>* rest, std::vector<std::string>* warnings, std::string* err);

// YAML file: unknown keys are returned in `unknown` (warned about, not fatal); bad values fail.
bool options_load_file(NativeOptions* o, const std::string& path, std::vector<std::string>* unknown, std::string* err);

// NODE_NAME, INFLUXDB_URL, GPUMON_<KEY> (GPUMON_CONFIG / GPUMON_AMDSMI_LIB excluded, as in Python).
// GPUMON_* variables that are neither a key nor an environment-only variable (a typo) go to
// `unknown` when given.
bool options_apply_env(NativeOptions* o, char** envp, std::string* err, std::vector<std::string>* unknown = nullptr);

// GPUMON_* variables read with getenv() by the runtime (tuning, diagnosis, library paths), which are
// not configuration keys (docs/configuration.md's environment-only table; the test fakes'
// GPUMON_FAKE_* are not listed).
const std::vector<std::string>& env_only_variables();

// Resolves listen / debug addresses, host name fallback, control-plane sockets (existence checks, CRI
// autodetect) and the on-device cadence into cfg / od (after all sources). false with *err for an
// address parse_listen / parse_debug_listen refuses.
bool options_finalize(NativeOptions* o, std::string* err);
const std::vector<std::string>& cri_autodetect_sockets();

// Checks a finalized configuration can run before anything starts (the Influx push, the /metrics
// TLS files, the bearer token file): "" or the reason (the binary exits 2 with it).
std::string options_validate(const NativeOptions& o);

int options_log_level(const NativeOptions& o);  // log_level -> g_log_level value

// Configuration as one JSON object keyed like the file (--print-config; the bindings read it
// unredacted).
std::string options_json(const NativeOptions& o, bool redact = true);

}  // namespace gpumon
