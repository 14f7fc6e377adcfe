// Standalone-binary configuration: YAML subset + env + flags, keyed like gpumon/config.py (options.h).
#include "options.h"

#include <unistd.h>

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <sstream>

#include "common.h"
#include "http_client.h"
#include "http_server.h"

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

Setter str(std::string NativeOptions::*m) {
  return [m](NativeOptions* o, const std::vector<std::string>& v, std::string*) {
    o->*m = v.empty() ? "" : v[0];
    return true;
  };
}
template <class F>
Setter str_at(F get) {
  return [get](NativeOptions* o, const std::vector<std::string>& v, std::string*) {
    *get(o) = v.empty() ? "" : v[0];
    return true;
  };
}
template <class F>
Setter bool_at(F get) {
  return [get](NativeOptions* o, const std::vector<std::string>& v, std::string* e) {
    return !v.empty() && to_bool(v[0], get(o), e);
  };
}
template <class F>
Setter int_at(F get) {
  return [get](NativeOptions* o, const std::vector<std::string>& v, std::string* e) {
    return !v.empty() && to_int(v[0], get(o), e);
  };
}
template <class F>
Setter dbl_at(F get) {
  return [get](NativeOptions* o, const std::vector<std::string>& v, std::string* e) {
    return !v.empty() && to_double(v[0], get(o), e);
  };
}
template <class F>
Setter list_at(F get) {
  return [get](NativeOptions* o, const std::vector<std::string>& v, std::string*) {
    *get(o) = as_list(v);
    return true;
  };
}

const std::map<std::string, Setter>& setters() {
  static const std::map<std::string, Setter> t = {
      {"backend", str_at([](NativeOptions* o) { return &o->cfg.backend; })},
      {"amdsmi_lib", str_at([](NativeOptions* o) { return &o->cfg.amdsmi_lib; })},
      {"rocm_smi_lib", str_at([](NativeOptions* o) { return &o->cfg.rocm_smi_lib; })},
      {"fast_path", bool_at([](NativeOptions* o) { return &o->cfg.fast_path; })},
      {"sysfs_root", str_at([](NativeOptions* o) { return &o->cfg.sysfs_root; })},
      {"devices",
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
       }},
      {"interval", dbl_at([](NativeOptions* o) { return &o->cfg.interval_s; })},
      {"processes", bool_at([](NativeOptions* o) { return &o->cfg.processes; })},
      {"link_every", int_at([](NativeOptions* o) { return &o->cfg.link_every; })},
      {"ras_every", int_at([](NativeOptions* o) { return &o->cfg.ras_every; })},
      {"ras_slices", int_at([](NativeOptions* o) { return &o->cfg.ras_slices; })},
      {"ras_async", bool_at([](NativeOptions* o) { return &o->cfg.ras_async; })},
      {"occ_samples", int_at([](NativeOptions* o) { return &o->cfg.occ_samples; })},
      {"prewarm_ms", dbl_at([](NativeOptions* o) { return &o->cfg.prewarm_ms; })},
      {"stale_hold_s", dbl_at([](NativeOptions* o) { return &o->cfg.stale_hold_s; })},
      {"hide_empty_contexts", bool_at([](NativeOptions* o) { return &o->cfg.hide_empty_contexts; })},
      {"mfma_exclusive_window_s", dbl_at([](NativeOptions* o) { return &o->cfg.mfma_exclusive_window_s; })},
      {"peer_context_max_vram_mib", dbl_at([](NativeOptions* o) { return &o->cfg.peer_context_max_vram_mib; })},
      {"sample_threads", int_at([](NativeOptions* o) { return &o->cfg.sample_threads; })},
      {"rt_priority", int_at([](NativeOptions* o) { return &o->cfg.rt_priority; })},
      {"device_timeout_s", dbl_at([](NativeOptions* o) { return &o->cfg.device_timeout_s; })},
      {"reinit_after", int_at([](NativeOptions* o) { return &o->cfg.reinit_after; })},
      {"init_retry_s", dbl_at([](NativeOptions* o) { return &o->cfg.init_retry_s; })},
      {"health_stale_s", dbl_at([](NativeOptions* o) { return &o->cfg.health_stale_s; })},
      {"listen", str(&NativeOptions::listen)},
      {"http_threads", int_at([](NativeOptions* o) { return &o->cfg.http_threads; })},
      {"http_rt_priority", int_at([](NativeOptions* o) { return &o->cfg.http_rt_priority; })},
      {"http_rt_budget", dbl_at([](NativeOptions* o) { return &o->cfg.http_rt_budget; })},
      {"host", str_at([](NativeOptions* o) { return &o->cfg.host; })},
      {"gzip", bool_at([](NativeOptions* o) { return &o->cfg.gzip; })},
      {"roctx", bool_at([](NativeOptions* o) { return &o->cfg.roctx; })},
      {"compat_families", bool_at([](NativeOptions* o) { return &o->cfg.compat_families; })},
      {"extended_families", bool_at([](NativeOptions* o) { return &o->cfg.extended_families; })},
      {"full_device_labels", bool_at([](NativeOptions* o) { return &o->cfg.full_device_labels; })},
      {"metrics_include", list_at([](NativeOptions* o) { return &o->cfg.metrics_include; })},
      {"metrics_exclude", list_at([](NativeOptions* o) { return &o->cfg.metrics_exclude; })},
      {"influx_url", str_at([](NativeOptions* o) { return &o->cfg.influx_url; })},
      {"influx_token", str_at([](NativeOptions* o) { return &o->cfg.influx_token; })},
      {"influx_extended", bool_at([](NativeOptions* o) { return &o->cfg.influx_extended; })},
      {"influx_schema", int_at([](NativeOptions* o) { return &o->cfg.influx_schema; })},
      {"influx_every", int_at([](NativeOptions* o) { return &o->cfg.influx_every; })},
      {"influx_gzip", bool_at([](NativeOptions* o) { return &o->cfg.influx_gzip; })},
      {"influx_ca_file", str_at([](NativeOptions* o) { return &o->cfg.influx_ca_file; })},
      {"tls_cert_file", str_at([](NativeOptions* o) { return &o->cfg.tls_cert_file; })},
      {"tls_key_file", str_at([](NativeOptions* o) { return &o->cfg.tls_key_file; })},
      {"tls_client_ca_file", str_at([](NativeOptions* o) { return &o->cfg.tls_client_ca_file; })},
      {"http_auth_token_file", str_at([](NativeOptions* o) { return &o->cfg.http_auth_token_file; })},
      {"influx_tls_insecure", bool_at([](NativeOptions* o) { return &o->cfg.influx_tls_insecure; })},
      {"influx_client_cert", str_at([](NativeOptions* o) { return &o->cfg.influx_client_cert; })},
      {"influx_client_key", str_at([](NativeOptions* o) { return &o->cfg.influx_client_key; })},
      {"procfs_root", str_at([](NativeOptions* o) { return &o->cfg.attribution.procfs_root; })},
      {"opt_in_label", str_at([](NativeOptions* o) { return &o->cfg.attribution.opt_in; })},
      {"user_label", str_at([](NativeOptions* o) { return &o->cfg.attribution.user_label; })},
      {"user_regex", str_at([](NativeOptions* o) { return &o->cfg.attribution.user_regex; })},
      {"user_prefix", str_at([](NativeOptions* o) { return &o->cfg.attribution.user_prefix; })},
      {"pod_label_allowlist", list_at([](NativeOptions* o) { return &o->cfg.attribution.label_allowlist; })},
      {"compat_user_rule", bool_at([](NativeOptions* o) { return &o->cfg.attribution.compat_user_rule; })},
      {"procfs_env_fallback", bool_at([](NativeOptions* o) { return &o->cfg.attribution.procfs_env_fallback; })},
      {"include_host_processes",
       bool_at([](NativeOptions* o) { return &o->cfg.attribution.include_host_processes; })},
      {"verify_kfd", bool_at([](NativeOptions* o) { return &o->cfg.attribution.verify_kfd; })},
      {"cri_socket", str(&NativeOptions::cri_socket)},
      {"docker_socket", str_at([](NativeOptions* o) { return &o->cfg.docker_socket; })},
      {"pod_log_root", str_at([](NativeOptions* o) { return &o->cfg.pod_log_root; })},
      {"device_checkpoint", str_at([](NativeOptions* o) { return &o->cfg.device_checkpoint; })},
      {"pod_resources_socket", str(&NativeOptions::pod_resources_socket)},
      {"resource_names", list_at([](NativeOptions* o) { return &o->resource_names; })},
      {"dra_drivers", list_at([](NativeOptions* o) { return &o->cfg.pod_resources_dra_drivers; })},
      {"metadata_refresh", dbl_at([](NativeOptions* o) { return &o->metadata_refresh_s; })},
      {"enable_probe", bool_at([](NativeOptions* o) { return &o->od.probe; })},
      {"probe_every", int_at([](NativeOptions* o) { return &o->probe_every; })},
      {"enable_pmc", bool_at([](NativeOptions* o) { return &o->od.pmc; })},
      {"pmc_counters", list_at([](NativeOptions* o) { return &o->od.pmc_counters; })},
      {"pmc_mode", str_at([](NativeOptions* o) { return &o->od.pmc_mode; })},
      {"ondevice_isolate", bool_at([](NativeOptions* o) { return &o->od.ondevice_isolate; })},
      {"helper_retry", dbl_at([](NativeOptions* o) { return &o->od.helper_retry_s; })},
      {"plugin_dir", str_at([](NativeOptions* o) { return &o->od.plugin_dir; })},
      {"activity_acc_scale", dbl_at([](NativeOptions* o) { return &o->cfg.rates.activity_acc_scale; })},
      {"xgmi_kb_bytes", dbl_at([](NativeOptions* o) { return &o->cfg.rates.xgmi_kb_bytes; })},
      {"log_level", str(&NativeOptions::log_level)},
  };
  return t;
}

void json_str(const std::string& s, std::string* o) {
  o->push_back('"');
  for (char c : s) {
    if (c == '"' || c == '\\') o->push_back('\\');
    if (c == '\n') {
      o->append("\\n");
      continue;
    }
    if (static_cast<unsigned char>(c) < 0x20) continue;
    o->push_back(c);
  }
  o->push_back('"');
}

}  // namespace

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
  const auto& t = setters();
  auto it = t.find(key);
  if (it == t.end()) return 0;
  std::string e;
  if (!it->second(o, vals, &e)) {
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

bool options_apply_env(NativeOptions* o, char** envp, std::string* err) {
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
    if (k == "CONFIG" || k == "AMDSMI_LIB" || k == "PLUGIN_DIR" || k == "ROCTX") continue;  // read where used
    for (auto& c : k) c = static_cast<char>(tolower(static_cast<unsigned char>(c)));
    std::string e;
    if (options_set(o, k, {kv.substr(eq + 1)}, &e) < 0) {
      *err = "GPUMON_" + kv.substr(7, eq - 7) + ": " + e;
      return false;
    }
  }
  return true;
}

bool options_finalize(NativeOptions* o, std::string* err) {
  ExporterConfig& c = o->cfg;
  if (!parse_listen(o->listen, &c.listen_addr, &c.port, err)) return false;
  if (c.host.empty()) c.host = "no_name";
  if (!o->resource_names.empty()) c.pod_resources_prefix = o->resource_names[0];
  c.pod_resources_refresh_s = o->metadata_refresh_s;
  if (!o->pod_resources_socket.empty() && o->pod_resources_socket != "none" &&
      access(o->pod_resources_socket.c_str(), F_OK) == 0)
    c.pod_resources_socket = o->pod_resources_socket;
  std::string cri = o->cri_socket;
  if (starts_with(cri, "unix://")) cri = cri.substr(7);
  if (cri.empty()) {
    for (const char* s : {"/run/containerd/containerd.sock", "/var/run/crio/crio.sock", "/run/crio/crio.sock",
                          "/var/run/cri-dockerd.sock", "/var/run/dockershim.sock"})
      if (access(s, F_OK) == 0) {
        cri = s;
        break;
      }
  }
  if (!cri.empty() && cri != "none") c.cri_socket = cri;
  const double period = c.interval_s > 0 ? std::max(c.interval_s, 0.1) : 1.0;
  o->od.pmc_every_s = period;
  o->od.probe_every_s = period * std::max(1, o->probe_every);
  const std::string& l = o->log_level;
  g_log_level = l == "debug" ? 0 : l == "info" ? 1 : (l == "warn" || l == "warning") ? 2 : l == "error" ? 3 : 1;
  return true;
}

std::string options_json(const NativeOptions& o) {
  const ExporterConfig& c = o.cfg;
  std::string s = "{";
  bool first = true;
  auto key = [&](const char* k) {
    if (!first) s += ", ";
    first = false;
    json_str(k, &s);
    s += ": ";
  };
  auto S = [&](const char* k, const std::string& v) {
    key(k);
    json_str(v, &s);
  };
  auto B = [&](const char* k, bool v) {
    key(k);
    s += v ? "true" : "false";
  };
  auto N = [&](const char* k, double v) {
    key(k);
    char b[64];
    snprintf(b, sizeof b, "%.17g", v);
    s += b;
  };
  auto L = [&](const char* k, const std::vector<std::string>& v) {
    key(k);
    s += "[";
    for (size_t i = 0; i < v.size(); ++i) {
      if (i) s += ", ";
      json_str(v[i], &s);
    }
    s += "]";
  };
  S("backend", c.backend);
  B("fast_path", c.fast_path);
  S("sysfs_root", c.sysfs_root);
  L("devices", c.devices);
  N("interval", c.interval_s);
  B("processes", c.processes);
  N("link_every", c.link_every);
  N("ras_every", c.ras_every);
  N("ras_slices", c.ras_slices);
  B("ras_async", c.ras_async);
  N("occ_samples", c.occ_samples);
  N("prewarm_ms", c.prewarm_ms);
  N("stale_hold_s", c.stale_hold_s);
  B("hide_empty_contexts", c.hide_empty_contexts);
  N("mfma_exclusive_window_s", c.mfma_exclusive_window_s);
  N("peer_context_max_vram_mib", c.peer_context_max_vram_mib);
  N("sample_threads", c.sample_threads);
  N("rt_priority", c.rt_priority);
  N("device_timeout_s", c.device_timeout_s);
  N("reinit_after", c.reinit_after);
  N("init_retry_s", c.init_retry_s);
  N("health_stale_s", c.health_stale_s);
  S("listen", o.listen);
  N("http_threads", c.http_threads);
  N("http_rt_priority", c.http_rt_priority);
  N("http_rt_budget", c.http_rt_budget);
  S("host", c.host);
  B("gzip", c.gzip);
  B("roctx", c.roctx);
  B("compat_families", c.compat_families);
  B("extended_families", c.extended_families);
  L("metrics_include", c.metrics_include);
  L("metrics_exclude", c.metrics_exclude);
  S("influx_url", redact_url(c.influx_url));
  S("influx_token", c.influx_token.empty() ? "" : "***");
  B("influx_extended", c.influx_extended);
  N("influx_schema", c.influx_schema);
  N("influx_every", c.influx_every);
  B("influx_gzip", c.influx_gzip);
  S("influx_ca_file", c.influx_ca_file);
  S("tls_cert_file", c.tls_cert_file);
  S("tls_key_file", c.tls_key_file);
  S("tls_client_ca_file", c.tls_client_ca_file);
  S("http_auth_token_file", c.http_auth_token_file);
  B("influx_tls_insecure", c.influx_tls_insecure);
  S("influx_client_cert", c.influx_client_cert);
  S("influx_client_key", c.influx_client_key);
  S("procfs_root", c.attribution.procfs_root);
  S("opt_in_label", c.attribution.opt_in);
  S("user_label", c.attribution.user_label);
  S("user_regex", c.attribution.user_regex);
  S("user_prefix", c.attribution.user_prefix);
  L("pod_label_allowlist", c.attribution.label_allowlist);
  B("compat_user_rule", c.attribution.compat_user_rule);
  B("procfs_env_fallback", c.attribution.procfs_env_fallback);
  B("include_host_processes", c.attribution.include_host_processes);
  S("cri_socket", o.cri_socket);
  S("docker_socket", c.docker_socket);
  S("pod_log_root", c.pod_log_root);
  S("device_checkpoint", c.device_checkpoint);
  S("pod_resources_socket", o.pod_resources_socket);
  L("resource_names", o.resource_names);
  L("dra_drivers", c.pod_resources_dra_drivers);
  N("metadata_refresh", o.metadata_refresh_s);
  B("enable_probe", o.od.probe);
  N("probe_every", o.probe_every);
  B("enable_pmc", o.od.pmc);
  L("pmc_counters", o.od.pmc_counters);
  S("pmc_mode", o.od.pmc_mode);
  B("ondevice_isolate", o.od.ondevice_isolate);
  N("helper_retry", o.od.helper_retry_s);
  S("plugin_dir", o.od.plugin_dir);
  N("activity_acc_scale", c.rates.activity_acc_scale);
  N("xgmi_kb_bytes", c.rates.xgmi_kb_bytes);
  S("log_level", o.log_level);
  s += "}";
  return s;
}

}  // namespace gpumon
