// The exporter configuration: YAML subset + env + flags, one key table for every entry point (options.h).
#include "options.h"

#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <sstream>

#include "common.h"
#include "http_auth.h"
#include "http_client.h"
#include "http_server.h"
#include "json_out.h"
#include "tls.h"

namespace gpumon {

namespace {

// ---------------------------------------------------------------------------------------------
// YAML subset

// Index of a comment '#' (start of line or after whitespace, outside quotes), or npos.
size_t comment_pos(const std::string& s) {
  char q = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (q) {
      if (c == '\\' && q == '"') ++i;
      else if (c == q) q = 0;
    } else if (c == '"' || c == '\'') {
      q = c;
    } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
      return i;
    }
  }
  return std::string::npos;
}

bool unquote(std::string v, std::string* out, std::string* err) {
  v = std::string(trim(v));
  if (v.size() >= 2 && v.front() == '\'' && v.back() == '\'') {
    out->clear();
    for (size_t i = 1; i + 1 < v.size(); ++i) {
      out->push_back(v[i]);
      if (v[i] == '\'' && i + 2 < v.size() && v[i + 1] == '\'') ++i;  // '' -> '
    }
    return true;
  }
  if (v.size() >= 2 && v.front() == '"' && v.back() == '"') {
    out->clear();
    for (size_t i = 1; i + 1 < v.size(); ++i) {
      char c = v[i];
      if (c == '\\' && i + 2 < v.size()) {
        c = v[++i];
        if (c == 'n') c = '\n';
        else if (c == 't') c = '\t';
      }
      out->push_back(c);
    }
    return true;
  }
  if (!v.empty() && (v.front() == '"' || v.front() == '\'')) {
    *err = "unterminated quoted value";
    return false;
  }
  if (!v.empty() && (v.front() == '{' || v.front() == '&' || v.front() == '*' || v.front() == '|' || v.front() == '>')) {
    *err = "unsupported YAML construct '" + v.substr(0, 1) + "' (flat key: value mapping only)";
    return false;
  }
  *out = v;
  return true;
}

bool split_flow_list(const std::string& body, std::vector<std::string>* out, std::string* err) {
  std::string cur;
  char q = 0;
  auto flush = [&]() -> bool {
    std::string v;
    if (!unquote(cur, &v, err)) return false;
    if (!trim(cur).empty()) out->push_back(v);
    cur.clear();
    return true;
  };
  for (size_t i = 0; i < body.size(); ++i) {
    const char c = body[i];
    if (q) {
      if (c == '\\' && q == '"' && i + 1 < body.size()) {
        cur.push_back(c);
        cur.push_back(body[++i]);
        continue;
      }
      if (c == q) q = 0;
      cur.push_back(c);
    } else if (c == '"' || c == '\'') {
      q = c;
      cur.push_back(c);
    } else if (c == ',') {
      if (!flush()) return false;
    } else if (c == '[' || c == '{') {
      *err = "nested collections are not supported";
      return false;
    } else {
      cur.push_back(c);
    }
  }
  if (q) {
    *err = "unterminated quoted value";
    return false;
  }
  return flush();
}

// ---------------------------------------------------------------------------------------------
// typed setters

bool to_bool(const std::string& v, bool* out, std::string* err) {
  std::string l;
  for (char c : v) l.push_back(static_cast<char>(tolower(static_cast<unsigned char>(c))));
  if (l == "1" || l == "true" || l == "yes" || l == "on") *out = true;
  else if (l == "0" || l == "false" || l == "no" || l == "off") *out = false;
  else {
    *err = "not a boolean: '" + v + "'";
    return false;
  }
  return true;
}

bool to_int(const std::string& v, int* out, std::string* err) {
  errno = 0;
  char* end = nullptr;
  const long x = strtol(v.c_str(), &end, 10);
  if (v.empty() || errno || *end) {
    *err = "not an integer: '" + v + "'";
    return false;
  }
  *out = static_cast<int>(x);
  return true;
}

bool to_double(const std::string& v, double* out, std::string* err) {
  errno = 0;
  char* end = nullptr;
  const double x = strtod(v.c_str(), &end);
  if (v.empty() || errno || *end || !std::isfinite(x)) {
    *err = "not a number: '" + v + "'";
    return false;
  }
  *out = x;
  return true;
}

// A list key given as one scalar (env var, or `key: a,b`) is split on commas, as in Python.
std::vector<std::string> as_list(const std::vector<std::string>& vals) {
  if (vals.size() != 1) return vals;
  std::vector<std::string> out;
  for (const auto& s : split(vals[0], ','))
    if (!trim(s).empty()) out.emplace_back(trim(s));
  return out;
}

using Setter = std::function<bool(NativeOptions*, const std::vector<std::string>&, std::string*)>;
using Getter = std::function<void(const NativeOptions&, JsonOut*, bool redact)>;

struct Key {
  OptionKey doc;
  Setter set;
  Getter get;
};

// Accessors take a mutable NativeOptions; the getters only read through them.
template <class F>
auto* at(const NativeOptions& o, F get) {
  return get(const_cast<NativeOptions*>(&o));
}

template <class F>
Key str_key(const char* k, const char* sec, const char* help, F get) {
  return {{k, sec, help},
          [get](NativeOptions* o, const std::vector<std::string>& v, std::string*) {
            *get(o) = v.empty() ? "" : v[0];
            return true;
          },
          [get](const NativeOptions& o, JsonOut* j, bool) { j->str(*at(o, get)); }};
}
template <class F>
Key bool_key(const char* k, const char* sec, const char* help, F get) {
  return {{k, sec, help},
          [get](NativeOptions* o, const std::vector<std::string>& v, std::string* e) {
            return !v.empty() && to_bool(v[0], get(o), e);
          },
          [get](const NativeOptions& o, JsonOut* j, bool) { j->boolean(*at(o, get)); }};
}
template <class F>
Key int_key(const char* k, const char* sec, const char* help, F get) {
  return {{k, sec, help},
          [get](NativeOptions* o, const std::vector<std::string>& v, std::string* e) {
            return !v.empty() && to_int(v[0], get(o), e);
          },
          [get](const NativeOptions& o, JsonOut* j, bool) { j->i64(*at(o, get)); }};
}
template <class F>
Key dbl_key(const char* k, const char* sec, const char* help, F get) {
  return {{k, sec, help},
          [get](NativeOptions* o, const std::vector<std::string>& v, std::string* e) {
            return !v.empty() && to_double(v[0], get(o), e);
          },
          [get](const NativeOptions& o, JsonOut* j, bool) { j->num(*at(o, get)); }};
}
template <class F>
Key list_key(const char* k, const char* sec, const char* help, F get) {
  return {{k, sec, help},
          [get](NativeOptions* o, const std::vector<std::string>& v, std::string*) {
            *get(o) = as_list(v);
            return true;
          },
          [get](const NativeOptions& o, JsonOut* j, bool) {
            j->arr();
            for (const auto& x : *at(o, get)) j->str(x);
            j->end_arr();
          }};
}

#define O(expr) [](NativeOptions* o) { return &(expr); }

constexpr const char* kBackend = "device backend";
constexpr const char* kExpo = "exposition";
constexpr const char* kPush = "influx compat push";
constexpr const char* kAttr = "attribution";
constexpr const char* kPlane = "control plane (k8s)";
constexpr const char* kOnDev = "on-device probe / PMC";
constexpr const char* kRates = "rates calibration";
constexpr const char* kLog = "logging";

// Every configuration key, in documentation order: the one table behind the YAML file, the
// GPUMON_<KEY> environment, the flags (option_flags), --print-config and the Python bindings
// (gpumon.config is a view of this, docs/configuration.md is generated from it).
const std::vector<Key>& keys() {
  static const std::vector<Key> t = {
      str_key("backend", kBackend, "auto / amdsmi / rocm_smi / mock[:k=v,...] (auto = libamd_smi, rocm_smi_lib if it cannot initialise)",
              O(o->cfg.backend)),
      str_key("amdsmi_lib", kBackend, "libamd_smi path tried first", O(o->cfg.amdsmi_lib)),
      str_key("rocm_smi_lib", kBackend, "librocm_smi64 override (rocm_smi backend / auto fallback)", O(o->cfg.rocm_smi_lib)),
      bool_key("fast_path", kBackend, "amdsmi: hot per-tick reads straight from sysfs/KFD", O(o->cfg.fast_path)),
      str_key("sysfs_root", kBackend, "sysfs mount (a host /sys bind-mounted elsewhere, or a test tree)", O(o->cfg.sysfs_root)),
      {{"devices", kBackend, "hip ids (\"3\") and / or PCI BDFs (\"0000:75:00.0\"); empty = every GPU"},
       [](NativeOptions* o, const std::vector<std::string>& v, std::string* e) {
         std::vector<std::string> ids;
         for (const auto& s : as_list(v)) {
           int x;
           std::string b = normalize_bdf(s);
           if (!b.empty()) {
             ids.push_back(b);
           } else if (to_int(s, &x, e) && x >= 0) {
             ids.push_back(std::to_string(x));
           } else {
             if (e) *e = "devices: '" + s + "' is neither a hip id nor a PCI BDF";
             return false;
           }
         }
         o->cfg.devices = ids;
         return true;
       },
       [](const NativeOptions& o, JsonOut* j, bool) {
         j->arr();
         for (const auto& x : o.cfg.devices) j->str(x);
         j->end_arr();
       }},
      dbl_key("interval", kBackend, "seconds; 0.1 = 10 Hz stress config (the reference slept 10 s, gpu.py:263)", O(o->cfg.interval_s)),
      bool_key("processes", kBackend, "list GPU processes (pod_gpu rows)", O(o->cfg.processes)),
      int_key("link_every", kBackend, "ticks between link-metrics refreshes (+ whenever a link's state changes)", O(o->cfg.link_every)),
      int_key("ras_every", kBackend, "ticks per full RAS / ECC pass (0 = off)", O(o->cfg.ras_every)),
      int_key("ras_slices", kBackend, "the pass read in this many slices on consecutive ticks (1..ras_every)", O(o->cfg.ras_slices)),
      bool_key("ras_async", kBackend, "device workers read RAS after publishing a tick (next tick carries it)", O(o->cfg.ras_async)),
      bool_key("hide_empty_contexts", kBackend, "no pod_gpu row for a GPU context with no VRAM and no waves", O(o->cfg.hide_empty_contexts)),
      dbl_key("mfma_exclusive_window_s", kBackend,
              "pod MFMA util only when no other process had waves in the last 5 ticks and this many seconds",
              O(o->cfg.mfma_exclusive_window_s)),
      dbl_key("peer_context_max_vram_mib", kBackend,
              "where KFD's per-process queue list cannot be read: a multi-GPU process's context on a GPU it does not "
              "work on (<= this VRAM, no waves, a workload on another GPU) gets no row. 0 = no peer-context "
              "hiding at all, the queue rule included",
              O(o->cfg.peer_context_max_vram_mib)),
      int_key("occ_samples", kBackend, "KFD cu_occupancy reads per process per tick (device workers; 1 = the tick's own)",
              O(o->cfg.occ_samples)),
      dbl_key("prewarm_ms", kBackend, "device workers warm the firmware-table path this long before each tick (0 = off)",
              O(o->cfg.prewarm_ms)),
      dbl_key("stale_hold_s", kBackend, "a repeated firmware table keeps the last rates only while it is this old (then: invalid)",
              O(o->cfg.stale_hold_s)),
      int_key("sample_threads", kBackend, "-1 = one worker per GPU (parallel + watchdog); 0 = sequential", O(o->cfg.sample_threads)),
      int_key("rt_priority", kBackend, "SCHED_FIFO priority of the sampler + device workers (needs CAP_SYS_NICE)", O(o->cfg.rt_priority)),
      dbl_key("device_timeout_s", kBackend, "a device call still running after this is exported as hung", O(o->cfg.device_timeout_s)),
      int_key("reinit_after", kBackend, "ticks with every GPU failing before the backend is re-initialised", O(o->cfg.reinit_after)),
      dbl_key("init_retry_s", kBackend, "backoff between backend init attempts", O(o->cfg.init_retry_s)),
      dbl_key("health_stale_s", kBackend, "/healthz 503 after this long without a tick (0 = max(3*interval, 10 s))", O(o->cfg.health_stale_s)),
      str_key("listen", kExpo, "host:port / [v6]:port / :port (every address, dual-stack; IPv4 if no IPv6)", O(o->listen)),
      int_key("http_threads", kExpo, "HTTP loop threads serving /metrics", O(o->cfg.http_threads)),
      int_key("http_rt_priority", kExpo, "SCHED_FIFO HTTP loops (CAP_SYS_NICE), each capped at http_rt_budget of a CPU",
              O(o->cfg.http_rt_priority)),
      dbl_key("http_rt_budget", kExpo, "share of a CPU per 100 ms an RT HTTP loop may use before it is demoted", O(o->cfg.http_rt_budget)),
      str_key("tls_cert_file", kExpo, "/metrics over HTTPS: PEM certificate chain (with tls_key_file)", O(o->cfg.tls_cert_file)),
      str_key("tls_key_file", kExpo, "... its PEM private key", O(o->cfg.tls_key_file)),
      str_key("tls_client_ca_file", kExpo,
              "mutual TLS: /metrics needs a client certificate signed by this CA (the health endpoints stay open "
              "for the kubelet's probes)",
              O(o->cfg.tls_client_ca_file)),
      str_key("http_auth_token_file", kExpo, "/metrics needs \"Authorization: Bearer <the file's token>\" (health endpoints stay open)",
              O(o->cfg.http_auth_token_file)),
      str_key("debug_listen", kExpo,
              "loopback-only JSON introspection (/debug/state, /debug/ticks, /debug/scrapes, ...) for benches and "
              "tests; \"\" = off",
              O(o->cfg.debug_listen)),
      str_key("host", kExpo, "node name label (default $NODE_NAME, then the host name, then \"no_name\")", O(o->cfg.host)),
      bool_key("gzip", kExpo, "gzip /metrics for scrapers that accept it", O(o->cfg.gzip)),
      bool_key("compat_families", kExpo, "serve the reference's node_gpu_* / pod_gpu_* families", O(o->cfg.compat_families)),
      bool_key("extended_families", kExpo, "serve the MI355X gpu_* families", O(o->cfg.extended_families)),
      bool_key("full_device_labels", kExpo, "uuid + bdf on every device series (default: on gpu_info only)", O(o->cfg.full_device_labels)),
      list_key("metrics_include", kExpo, "serve only families matching these globs (e.g. node_gpu_*)", O(o->cfg.metrics_include)),
      list_key("metrics_exclude", kExpo, "drop families matching these globs (e.g. gpu_xcd_*); Influx unfiltered", O(o->cfg.metrics_exclude)),
      {{"influx_url", kPush, "http(s)://[user:password@]host[:port]/path?query; checked at startup (exit 2 if unusable)"},
       [](NativeOptions* o, const std::vector<std::string>& v, std::string*) {
         o->cfg.influx_url = v.empty() ? "" : v[0];
         return true;
       },
       [](const NativeOptions& o, JsonOut* j, bool redact) { j->str(redact ? redact_url(o.cfg.influx_url) : o.cfg.influx_url); }},
      {{"influx_token", kPush, "InfluxDB 2.x/3.x API token (env INFLUXDB_TOKEN, from a Secret); 1.x: user:password@ in the URL"},
       [](NativeOptions* o, const std::vector<std::string>& v, std::string*) {
         o->cfg.influx_token = v.empty() ? "" : v[0];
         return true;
       },
       [](const NativeOptions& o, JsonOut* j, bool redact) {
         j->str(redact && !o.cfg.influx_token.empty() ? std::string("***") : o.cfg.influx_token);
       }},
      bool_key("influx_extended", kPush,
               "also push a gpu_ext line per GPU: UMC activity, hotspot / HBM temperature, power, energy, "
               "clocks, interval PCIe bytes/s and power, per-XCD busy, RAS totals",
               O(o->cfg.influx_extended)),
      int_key("influx_schema", kPush, "2019 = gpu.py layout; 2018 = img/influxdb.png pod_gpu layout", O(o->cfg.influx_schema)),
      int_key("influx_every", kPush, "ticks per push", O(o->cfg.influx_every)),
      dbl_key("influx_timeout_s", kPush, "seconds a push may take (connect, TLS handshake, request, answer) before it "
              "counts as failed and the batch is requeued", O(o->cfg.influx_timeout_s)),
      bool_key("influx_gzip", kPush, "gzip each push (Content-Encoding: gzip): 7-8x fewer bytes for 8 GPUs", O(o->cfg.influx_gzip)),
      str_key("influx_ca_file", kPush, "https:// push: PEM CA bundle replacing the system one", O(o->cfg.influx_ca_file)),
      bool_key("influx_tls_insecure", kPush, "https:// push WITHOUT certificate / host-name checks (opt-in, testing)",
               O(o->cfg.influx_tls_insecure)),
      str_key("influx_client_cert", kPush, "https:// push: PEM client chain for mutual TLS", O(o->cfg.influx_client_cert)),
      str_key("influx_client_key", kPush, "... and its key (default: in the chain file)", O(o->cfg.influx_client_key)),
      str_key("procfs_root", kAttr, "/proc of the host (hostPID)", O(o->cfg.attribution.procfs_root)),
      str_key("opt_in_label", kAttr, "only report pods with this label KEY=VALUE (reference: mlgpu=mlgpu, gpu.py:186-188)",
              O(o->cfg.attribution.opt_in)),
      str_key("user_label", kAttr, "pod label holding the user name", O(o->cfg.attribution.user_label)),
      str_key("user_regex", kAttr, "regex on the pod name; group 1 = user", O(o->cfg.attribution.user_regex)),
      list_key("pod_label_allowlist", kAttr,
               "pod / container label keys copied onto pod_gpu_* series as label_<key> (kube-state-metrics style)",
               O(o->cfg.attribution.label_allowlist)),
      str_key("user_prefix", kAttr, "pod-name prefix of the reference's user rule (gpu.py:196)", O(o->cfg.attribution.user_prefix)),
      bool_key("compat_user_rule", kAttr, "the reference's user-name rule when no label / regex names the user",
               O(o->cfg.attribution.compat_user_rule)),
      bool_key("procfs_env_fallback", kAttr, "pod name / namespace from the process's HOSTNAME and service-account files",
               O(o->cfg.attribution.procfs_env_fallback)),
      bool_key("include_host_processes", kAttr, "GPU processes outside any container get rows too",
               O(o->cfg.attribution.include_host_processes)),
      bool_key("verify_kfd", kAttr, "trust /proc/<pid> only when it holds /dev/kfd (guards a foreign pid namespace)",
               O(o->cfg.attribution.verify_kfd)),
      {{"control_plane", kPlane, "native: the kubelet PodResources / CRI / Docker / log-tree pollers; off: none of them"},
       [](NativeOptions* o, const std::vector<std::string>& v, std::string* e) {
         const std::string x = v.empty() ? "" : v[0];
         if (x != "native" && x != "off") {
           *e = "native or off, not '" + x + "'";
           return false;
         }
         o->control_plane = x;
         return true;
       },
       [](const NativeOptions& o, JsonOut* j, bool) { j->str(o.control_plane); }},
      str_key("cri_socket", kPlane, "e.g. unix:///run/containerd/containerd.sock; \"\" = autodetect; none = off", O(o->cri_socket)),
      str_key("pod_resources_socket", kPlane, "kubelet PodResources socket (idle-allocation rows); \"\" = off",
              O(o->pod_resources_socket)),
      str_key("docker_socket", kPlane, "plain-Docker nodes: Docker Engine container names + labels; opt-in, e.g. /var/run/docker.sock",
              O(o->cfg.docker_socket)),
      str_key("pod_log_root", kPlane, "non-root metadata: the kubelet's log tree (containers/ + pods/ under it), e.g. /var/log; \"\" = off",
              O(o->cfg.pod_log_root)),
      str_key("device_checkpoint", kPlane,
              "GPU allocations from the kubelet's device-plugin checkpoint, e.g. "
              "/var/lib/kubelet/device-plugins/kubelet_internal_checkpoint; \"\" = off",
              O(o->cfg.device_checkpoint)),
      list_key("resource_names", kPlane, "extended resources that are GPUs (the first one is counted)", O(o->resource_names)),
      {{"dra_drivers", kPlane, "DRA drivers whose claimed devices count as GPU allocations ('none' or [] = off)"},
       [](NativeOptions* o, const std::vector<std::string>& v, std::string*) {
         auto l = as_list(v);
         if (l.size() == 1 && l[0] == "none") l.clear();
         o->cfg.pod_resources_dra_drivers = l;
         return true;
       },
       [](const NativeOptions& o, JsonOut* j, bool) {
         j->arr();
         for (const auto& x : o.cfg.pod_resources_dra_drivers) j->str(x);
         j->end_arr();
       }},
      dbl_key("metadata_refresh", kPlane, "seconds between control-plane refreshes", O(o->metadata_refresh_s)),
      bool_key("enable_probe", kOnDev, "K1 gfx950 probe kernel (per-XCD clock / liveness / dispatch latency)", O(o->od.probe)),
      int_key("probe_every", kOnDev, "K1 probe every N sampling intervals", O(o->probe_every)),
      int_key("probe_blocks", kOnDev, "one-wave workgroups per probe launch (>= 4 per CU spreads over all 8 XCDs)",
              O(o->od.probe_blocks)),
      bool_key("enable_pmc", kOnDev, "rocprofiler-sdk device counting (MFMA utilisation, TFLOP/s per dtype)", O(o->od.pmc)),
      list_key("pmc_counters", kOnDev,
               "counters of the PMC derivation (8 SQ + 2 GRBM: one gfx950 counting pass): MFMA busy + MOPS per operand type",
               O(o->od.pmc_counters)),
      str_key("pmc_mode", kOnDev,
              "continuous: counting contexts read without a stop (100 % of each interval); window: start -> pmc_window -> stop",
              O(o->od.pmc_mode)),
      dbl_key("pmc_window", kOnDev, "window mode: counting window per sample in seconds (capped at half the period)",
              O(o->od.pmc_window_s)),
      bool_key("ondevice_isolate", kOnDev,
               "the counting contexts and the probe in a helper process frozen between reads (rocprofiler-sdk leaves an "
               "HSA thread polling a full core in the process that owns them)",
               O(o->od.ondevice_isolate)),
      dbl_key("helper_retry", kOnDev, "seconds before a dead helper is respawned (doubling while it keeps dying)", O(o->od.helper_retry_s)),
      str_key("plugin_dir", kOnDev, "directory holding libgpumon_pmc.so / libgpumon_probe.so (\"\" = <tree>/lib or $GPUMON_PLUGIN_DIR)",
              O(o->od.plugin_dir)),
      dbl_key("activity_acc_scale", kRates, "avg % = d(activity acc) / d(accumulation_counter) x this", O(o->cfg.rates.activity_acc_scale)),
      dbl_key("xgmi_kb_bytes", kRates, "bytes per xGMI \"KB\" accumulator unit", O(o->cfg.rates.xgmi_kb_bytes)),
      dbl_key("pcie_bw_unit_bytes", kRates,
              "bytes/s per firmware PCIe bandwidth unit (102400 measured on MI355X against pinned host copies)",
              O(o->cfg.rates.pcie_bw_unit_bytes)),
      str_key("log_level", kLog, "debug / info / warn / error", O(o->log_level)),
      bool_key("roctx", kLog, "ROCTx ranges around the sampler phases (rocprofv3 --marker-trace)", O(o->cfg.roctx)),
      // a key of earlier releases (it selected the Python test oracles): accepted, no effect
      {{"ondevice", "", ""},
       [](NativeOptions*, const std::vector<std::string>&, std::string*) { return true; },
       nullptr},
  };
  return t;
}

#undef O

const Key* find_key(const std::string& k) {
  static const std::map<std::string, const Key*> idx = [] {
    std::map<std::string, const Key*> m;
    for (const auto& x : keys()) m[x.doc.key] = &x;
    return m;
  }();
  auto it = idx.find(k);
  return it == idx.end() ? nullptr : it->second;
}

}  // namespace

const std::vector<OptionKey>& option_keys() {
  static const std::vector<OptionKey> v = [] {
    std::vector<OptionKey> out;
    for (const auto& k : keys())
      if (k.get) out.push_back(k.doc);
    return out;
  }();
  return v;
}

const std::vector<OptionFlag>& option_flags() {
  // {flag, aliases, key, fixed value (nullptr: the flag takes one), help}
  static const std::vector<OptionFlag> t = {
      {"--backend", "", "backend", nullptr, "auto | amdsmi | rocm_smi | mock[:k=v,..]"},
      {"--devices", "", "devices", nullptr, "comma-separated hip ids and / or PCI BDFs to monitor (default all)"},
      {"--interval", "", "interval", nullptr, "sampling interval in seconds"},
      {"--listen", "", "listen", nullptr, "HOST:PORT, [V6]:PORT or :PORT for /metrics"},
      {"--host", "", "host", nullptr, "node name label (default $NODE_NAME, then the host name)"},
      {"--no-fast-path", "", "fast_path", "false", "amdsmi: read every value through libamd_smi"},
      {"--sysfs-root", "--sysfs", "sysfs_root", nullptr, "sysfs mount"},
      {"--procfs-root", "--procfs", "procfs_root", nullptr, "procfs mount of the host"},
      {"--no-processes", "", "processes", "false", "no process list (no pod_gpu rows)"},
      {"--ras-every", "", "ras_every", nullptr, "RAS error counters every N ticks"},
      {"--ras-slices", "", "ras_slices", nullptr, "RAS blocks read in N slices over N ticks"},
      {"--device-timeout", "", "device_timeout_s", nullptr, "seconds before a device call is exported as hung"},
      {"--sample-threads", "", "sample_threads", nullptr, "per-GPU sampling threads (-1 = one per GPU, 0 = sequential)"},
      {"--rt-priority", "", "rt_priority", nullptr, "SCHED_FIFO priority of the sampler (0 = normal)"},
      {"--prewarm-ms", "", "prewarm_ms", nullptr, "warm the firmware-table read this long before each tick (0 = off)"},
      {"--occ-samples", "", "occ_samples", nullptr, "KFD cu_occupancy reads per process per tick (1 = the tick's own)"},
      {"--http-threads", "", "http_threads", nullptr, "HTTP loop threads serving /metrics"},
      {"--http-rt-priority", "", "http_rt_priority", nullptr, "SCHED_FIFO priority of the HTTP loops (0 = normal)"},
      {"--tls-cert-file", "", "tls_cert_file", nullptr, "serve /metrics over HTTPS: PEM certificate chain"},
      {"--tls-key-file", "", "tls_key_file", nullptr, "... and its PEM private key"},
      {"--tls-client-ca-file", "", "tls_client_ca_file", nullptr, "mutual TLS on /metrics: clients need a certificate signed by this CA"},
      {"--http-auth-token-file", "", "http_auth_token_file", nullptr, "/metrics needs 'Authorization: Bearer <token>' from this file"},
      {"--debug-listen", "", "debug_listen", nullptr, "loopback HOST:PORT for the JSON introspection endpoints"},
      {"--no-gzip", "", "gzip", "false", "never gzip /metrics"},
      {"--metrics-include", "", "metrics_include", nullptr, "comma-separated globs: serve only these families"},
      {"--metrics-exclude", "", "metrics_exclude", nullptr, "comma-separated globs: families left out of /metrics"},
      {"--influx-url", "", "influx_url", nullptr, "enable the InfluxDB line-protocol push (default $INFLUXDB_URL)"},
      {"--influx-token", "", "influx_token", nullptr, "InfluxDB 2.x / 3.x API token (default $INFLUXDB_TOKEN)"},
      {"--influx-extended", "", "influx_extended", "true", "also push the MI355X fields"},
      {"--influx-gzip", "", "influx_gzip", "true", "gzip each push"},
      {"--influx-schema", "", "influx_schema", nullptr, "pod_gpu line layout: 2019 (gpu.py) or 2018 (img/influxdb.png)"},
      {"--influx-ca-file", "", "influx_ca_file", nullptr, "PEM CA bundle for an https:// INFLUXDB_URL"},
      {"--influx-tls-insecure", "", "influx_tls_insecure", "true", "do NOT verify the InfluxDB server's certificate (testing only)"},
      {"--influx-client-cert", "", "influx_client_cert", nullptr, "PEM client certificate for the push (mutual TLS)"},
      {"--influx-client-key", "", "influx_client_key", nullptr, "PEM client key for the push"},
      {"--opt-in-label", "", "opt_in_label", nullptr, "only report pods with label KEY=VALUE"},
      {"--user-regex", "", "user_regex", nullptr, "regex on the pod name; group 1 = user"},
      {"--user-label", "", "user_label", nullptr, "pod label holding the user name"},
      {"--pod-labels", "", "pod_label_allowlist", nullptr, "comma-separated pod label keys exported as label_<key>"},
      {"--control-plane", "", "control_plane", nullptr, "native | off: the kubelet / CRI / Docker metadata pollers"},
      {"--cri-socket", "--cri", "cri_socket", nullptr, "CRI runtime socket (default: autodetect)"},
      {"--no-cri", "", "cri_socket", "none", "no CRI runtime lookup"},
      {"--pod-resources-socket", "--pod-resources", "pod_resources_socket", nullptr, "kubelet PodResources socket"},
      {"--no-pod-resources", "", "pod_resources_socket", "", "no kubelet PodResources polling (no idle-allocation rows)"},
      {"--docker-socket", "--docker", "docker_socket", nullptr, "plain-Docker nodes: the Docker Engine socket (opt-in)"},
      {"--pod-log-root", "--pod-logs", "pod_log_root", nullptr, "non-root metadata: the kubelet's log tree, e.g. /var/log"},
      {"--device-checkpoint", "", "device_checkpoint", nullptr, "GPU allocations from the device-plugin checkpoint file"},
      {"--dra-drivers", "", "dra_drivers", nullptr, "comma-separated DRA driver names ('none' = off)"},
      {"--enable-pmc", "--pmc", "enable_pmc", "true", "rocprofiler-sdk device counting (MFMA utilisation, TFLOP/s)"},
      {"--pmc-counters", "", "pmc_counters", nullptr, "comma-separated PMC counters"},
      {"--pmc-mode", "", "pmc_mode", nullptr, "continuous | window"},
      {"--pmc-window", "", "pmc_window", nullptr, "window mode: counting window in seconds"},
      {"--enable-probe-kernel", "--probe", "enable_probe", "true", "the K1 gfx950 probe kernel"},
      {"--probe-every", "", "probe_every", nullptr, "K1 probe every N ticks"},
      {"--probe-blocks", "", "probe_blocks", nullptr, "one-wave workgroups per probe launch"},
      {"--plugin-dir", "", "plugin_dir", nullptr, "directory holding libgpumon_pmc.so / libgpumon_probe.so"},
      {"--roctx", "", "roctx", "true", "bracket the sampler phases with ROCTx ranges"},
      {"--log-level", "", "log_level", nullptr, "debug | info | warn | error"},
  };
  return t;
}

bool parse_yaml_subset(const std::string& text, YamlDoc* doc, std::string* err) {

  std::istringstream in(text);
  std::string line, pending;  // pending: key awaiting block-list items
  int lineno = 0, base_indent = -1, top_indent = -1;
  bool in_top = false;
  while (std::getline(in, line)) {
    ++lineno;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    const size_t cp = comment_pos(line);
    if (cp != std::string::npos) line.resize(cp);
    if (trim(line).empty()) continue;
    if (line.find('\t') < line.find_first_not_of(" \t")) {
      *err = "line " + std::to_string(lineno) + ": tab indentation";
      return false;
    }
    const int indent = static_cast<int>(line.find_first_not_of(' '));
    const std::string content(trim(line));
    auto fail = [&](const std::string& m) {
      *err = "line " + std::to_string(lineno) + ": " + m;
      return false;
    };
    if (content == "---") continue;
    if (content[0] == '-' && (content.size() == 1 || content[1] == ' ')) {
      if (pending.empty()) return fail("list item without a key");
      std::string v, e;
      if (!unquote(content.substr(1), &v, &e)) return fail(e);
      doc->values[pending].push_back(v);
      continue;
    }
    size_t colon = std::string::npos;
    for (size_t i = 0; i < content.size(); ++i)
      if (content[i] == ':' && (i + 1 == content.size() || content[i + 1] == ' ')) {
        colon = i;
        break;
      }
    if (colon == std::string::npos || colon == 0) return fail("expected 'key: value'");
    const std::string key(trim(content.substr(0, colon)));
    const std::string rest(trim(content.substr(colon + 1)));
    if (key == "gpumon" && rest.empty() && doc->order.empty() && !in_top) {
      in_top = true;
      top_indent = indent;
      pending.clear();
      continue;
    }
    if (in_top && indent <= top_indent) return fail("only the 'gpumon:' mapping is allowed at the top level");
    if (base_indent < 0) base_indent = indent;
    if (indent != base_indent) return fail("nested mappings are not supported ('" + key + "')");
    if (doc->values.count(key)) return fail("duplicate key '" + key + "'");
    doc->order.push_back(key);
    auto& vals = doc->values[key];
    pending.clear();
    if (rest.empty()) {
      pending = key;  // block list follows (or an empty value)
    } else if (rest.front() == '[') {
      if (rest.back() != ']') return fail("unterminated flow list");
      std::string e;
      if (!split_flow_list(rest.substr(1, rest.size() - 2), &vals, &e)) return fail(e);
    } else {
      std::string v, e;
      if (!unquote(rest, &v, &e)) return fail(e);
      vals.push_back(v);
    }
  }
  return true;
}

int options_set(NativeOptions* o, const std::string& key, const std::vector<std::string>& vals, std::string* err) {
  const Key* k = find_key(key);
  if (!k) return 0;
  std::string e;
  if (!k->set(o, vals, &e)) {
    *err = key + ": " + (e.empty() ? "missing value" : e);
    return -1;
  }
  return 1;
}

bool options_load_file(NativeOptions* o, const std::string& path, std::vector<std::string>* unknown,
                       std::string* err) {
  std::string text;
  if (!read_file(path, &text, 1 << 20)) {
    *err = "cannot read " + path;
    return false;
  }
  YamlDoc doc;
  std::string e;
  if (!parse_yaml_subset(text, &doc, &e)) {
    *err = path + ": " + e;
    return false;
  }
  for (const auto& k : doc.order) {
    const int r = options_set(o, k, doc.values[k], &e);
    if (r < 0) {
      *err = path + ": " + e;
      return false;
    }
    if (r == 0 && unknown) unknown->push_back(k);
  }
  return true;
}

const std::vector<std::string>& env_only_variables() {
  static const std::vector<std::string> v = {
      "GPUMON_CONFIG",         "GPUMON_AMDSMI_LIB",      "GPUMON_ROCM_SMI_LIB",   "GPUMON_TLS_RELOAD_S",
      "GPUMON_HTTP_SNDBUF",    "GPUMON_LIBSSL",          "GPUMON_LIBCRYPTO",      "GPUMON_HTTP_HEADER_TIMEOUT_S",
      "GPUMON_HTTP_MEMORY_BUDGET", "GPUMON_ROCTX",       "GPUMON_PLUGIN_DIR",     "GPUMON_PROBE_RUNTIME",
      "GPUMON_PROBE_STREAM",   "GPUMON_PROBE_KERNARG",   "GPUMON_PMC_DEBUG_INIT", "GPUMON_LOAD_SYNC"};
  return v;
}

bool options_apply_env(NativeOptions* o, char** envp, std::string* err, std::vector<std::string>* unknown) {
  for (char** p = envp; p && *p; ++p) {
    const std::string kv = *p;
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    const std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
    if (k == "NODE_NAME" && !v.empty()) o->cfg.host = v;
    else if (k == "INFLUXDB_URL" && !v.empty()) o->cfg.influx_url = v;
    else if (k == "INFLUXDB_TOKEN" && !v.empty()) o->cfg.influx_token = v;
  }
  for (char** p = envp; p && *p; ++p) {
    const std::string kv = *p;
    const size_t eq = kv.find('=');
    if (eq == std::string::npos || !starts_with(kv, "GPUMON_")) continue;
    std::string k = kv.substr(7, eq - 7);
    // the file name itself, and an extra library path the backend tries after amdsmi_lib
    if (k == "CONFIG" || k == "AMDSMI_LIB") continue;
    for (auto& c : k) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
    std::string e;
    const int r = options_set(o, k, {kv.substr(eq + 1)}, &e);
    if (r < 0) {
      *err = "GPUMON_" + kv.substr(7, eq - 7) + ": " + e;
      return false;
    }
    const std::string name = kv.substr(0, eq);
    // Kubernetes service links of a Service named "gpumon" (GPUMON_SERVICE_HOST, GPUMON_PORT,
    // GPUMON_PORT_9400_TCP_ADDR, ...) when a pod spec leaves enableServiceLinks on: not ours
    const bool service_link =
        starts_with(name, "GPUMON_SERVICE_") || name == "GPUMON_PORT" || starts_with(name, "GPUMON_PORT_");
    if (r == 0 && unknown && !starts_with(name, "GPUMON_FAKE_") && !service_link) {
      const auto& known = env_only_variables();
      if (std::find(known.begin(), known.end(), name) == known.end()) unknown->push_back(name);
    }
  }
  return true;
}

const OptionFlag* find_flag(const std::string& arg) {
  for (const auto& f : option_flags()) {
    if (arg == f.flag) return &f;
    for (const auto& a : split(f.aliases, ','))
      if (!a.empty() && arg == a) return &f;
  }
  return nullptr;
}

ParseStatus options_parse(NativeOptions* o, const std::vector<std::string>& args, char** envp,
                          std::vector<std::string>* rest, std::vector<std::string>* warnings, std::string* err) {
  // 1. the file: --config wins over GPUMON_CONFIG
  std::string config;
  for (char** p = envp; p && *p; ++p)
    if (starts_with(*p, "GPUMON_CONFIG=")) config = *p + strlen("GPUMON_CONFIG=");
  bool compat = false;
  for (size_t i = 0; i < args.size(); ++i) {
    if (args[i] == "--config") {
      if (i + 1 >= args.size()) {
        *err = "--config: missing value";
        return ParseStatus::kBadFlag;
      }
      config = args[++i];
    } else if (starts_with(args[i], "--config=")) {
      config = args[i].substr(9);
      if (config.empty()) {
        *err = "--config: missing value";
        return ParseStatus::kBadFlag;
      }
    }
    else if (args[i] == "--compat") compat = true;
  }
  if (!config.empty()) {
    std::vector<std::string> unknown;
    if (!options_load_file(o, config, &unknown, err)) return ParseStatus::kBadFile;
    if (warnings)
      for (const auto& k : unknown) warnings->push_back("config: key '" + k + "' is not a configuration key (ignored)");
  }
  // 2. the environment
  std::vector<std::string> unknown_env;
  if (!options_apply_env(o, envp, err, &unknown_env)) return ParseStatus::kBadEnv;
  if (warnings)
    for (const auto& k : unknown_env)
      warnings->push_back("environment: " + k + " is neither a configuration key nor a GPUMON_ variable (ignored)");
  // 3. --compat (the reference's behaviour: opt-in label mlgpu=mlgpu, 10 s interval) between the
  // environment and the flags: explicit flags still win
  if (compat) {
    if (o->cfg.attribution.opt_in.empty()) o->cfg.attribution.opt_in = "mlgpu=mlgpu";
    o->cfg.interval_s = 10.0;
  }
  // 4. the flags, in order
  for (size_t i = 0; i < args.size(); ++i) {
    std::string a = args[i], val;
    bool inline_val = false;
    if (a == "--config") {
      ++i;
      continue;
    }
    if (a == "--compat" || starts_with(a, "--config=")) continue;
    const size_t eq = starts_with(a, "--") ? a.find('=') : std::string::npos;
    if (eq != std::string::npos) {
      val = a.substr(eq + 1);
      a = a.substr(0, eq);
      inline_val = true;
    }
    const OptionFlag* f = find_flag(a);
    if (!f) {
      if (!rest) {
        *err = "unknown flag " + args[i];
        return ParseStatus::kBadFlag;
      }
      rest->push_back(args[i]);
      continue;
    }
    if (f->fixed) {
      if (inline_val) {
        *err = a + " takes no value";
        return ParseStatus::kBadFlag;
      }
      val = f->fixed;
    } else if (!inline_val) {
      if (i + 1 >= args.size()) {
        *err = a + ": missing value";
        return ParseStatus::kBadFlag;
      }
      val = args[++i];
    }
    std::string e;
    if (options_set(o, f->key, {val}, &e) < 0) {
      *err = a + ": " + e.substr(e.find(": ") == std::string::npos ? 0 : e.find(": ") + 2);
      return ParseStatus::kBadValue;
    }
  }
  return ParseStatus::kOk;
}

// Well-known CRI runtime sockets, first existing one wins ("" cri_socket = autodetect).
static const char* const kCriSockets[] = {"/run/containerd/containerd.sock", "/var/run/containerd/containerd.sock",
                                          "/var/run/crio/crio.sock",         "/run/crio/crio.sock",
                                          "/var/run/cri-dockerd.sock",       "/var/run/dockershim.sock"};

const std::vector<std::string>& cri_autodetect_sockets() {
  static const std::vector<std::string> v(std::begin(kCriSockets), std::end(kCriSockets));
  return v;
}

bool options_finalize(NativeOptions* o, std::string* err) {
  ExporterConfig& c = o->cfg;
  if (!parse_listen(o->listen, &c.listen_addr, &c.port, err)) return false;
  if (!c.debug_listen.empty()) {
    std::string h;
    int p = 0;
    if (!parse_debug_listen(c.debug_listen, &h, &p, err)) return false;
  }
  // host: NODE_NAME (options_apply_env) > the machine's host name > the reference's "no_name"
  // (gpu.py:23-24, which never reached its lines: quirk Q1)
  if (c.host.empty()) {
    char hn[256] = {0};
    c.host = gethostname(hn, sizeof hn - 1) == 0 && hn[0] ? hn : "no_name";
  }
  if (!o->resource_names.empty()) c.pod_resources_prefix = o->resource_names[0];
  c.pod_resources_refresh_s = o->metadata_refresh_s;
  c.pod_resources_socket.clear();
  c.cri_socket.clear();
  if (o->control_plane == "off") {
    // no kubelet / CRI / Docker / log-tree metadata pollers
    c.docker_socket.clear();
    c.pod_log_root.clear();
    c.device_checkpoint.clear();
  } else {
    if (!o->pod_resources_socket.empty() && o->pod_resources_socket != "none" &&
        access(o->pod_resources_socket.c_str(), F_OK) == 0)
      c.pod_resources_socket = o->pod_resources_socket;
    std::string cri = o->cri_socket;
    if (starts_with(cri, "unix://")) cri = cri.substr(7);
    if (cri.empty())
      for (const auto& s : cri_autodetect_sockets())
        if (access(s.c_str(), F_OK) == 0) {
          cri = s;
          break;
        }
    if (!cri.empty() && cri != "none") c.cri_socket = cri;
    if (starts_with(c.docker_socket, "unix://")) c.docker_socket = c.docker_socket.substr(7);
  }
  const double period = c.interval_s > 0 ? std::max(c.interval_s, 0.1) : 1.0;
  o->od.pmc_every_s = period;
  o->od.probe_every_s = period * std::max(1, o->probe_every);
  return true;
}

int options_log_level(const NativeOptions& o) {
  const std::string& l = o.log_level;
  return l == "debug" ? 0 : l == "info" ? 1 : (l == "warn" || l == "warning") ? 2 : l == "error" ? 3 : l == "off" ? 4 : 1;
}

std::string options_validate(const NativeOptions& o) {
  const ExporterConfig& cfg = o.cfg;
  // an Influx push that cannot work is a startup error, not a silently idle pusher
  TlsOptions t;
  t.ca_file = cfg.influx_ca_file;
  t.insecure = cfg.influx_tls_insecure;
  t.client_cert = cfg.influx_client_cert;
  t.client_key = cfg.influx_client_key;
  std::string e = check_push_config(cfg.influx_url, cfg.influx_token, t);
  if (!e.empty()) return e;
  // /metrics over HTTPS: the certificate, key and client CA must load
  e = check_serve_tls(cfg.tls_cert_file, cfg.tls_key_file, cfg.tls_client_ca_file);
  if (!e.empty()) return e;
  // /metrics behind a bearer token: the token file must hold one
  e = check_auth_token_file(cfg.http_auth_token_file);
  if (!e.empty()) return "http_auth_token_file: " + e;
  if (o.od.pmc_mode != "continuous" && o.od.pmc_mode != "window") return "pmc_mode: continuous or window, not '" + o.od.pmc_mode + "'";
  return "";
}

std::string options_json(const NativeOptions& o, bool redact) {
  JsonOut j;
  j.obj();
  for (const auto& k : keys())
    if (k.get) {
      j.key(k.doc.key);
      k.get(o, &j, redact);
    }
  j.end_obj();
  return j.take();
}

}  // namespace gpumon
