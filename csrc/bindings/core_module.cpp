// pybind11 bindings: gpumon._core
//
// The Python control plane (config, CLI, CRI / PodResources clients, probe/PMC plugins, bench)
// drives the C++ core through this module. Every blocking call releases the GIL; the sampler,
// renderer and HTTP server never take it.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <set>
#include <thread>

#include "../core/attribution.h"
#include "../core/backend.h"
#include "../core/common.h"
#include "../core/docker_lite.h"
#include "../core/exporter.h"
#include "../core/grpc_lite.h"
#include "../core/hpack.h"
#include "../core/http_client.h"
#include "../core/kubelet_files.h"
#include "../core/ondevice.h"
#include "../core/options.h"
#include "../core/render.h"
#include "../core/snapshot.h"
#include "../core/trace.h"
#include "../core/sysfs_fast.h"
#include "../core/xgmi_map.h"

namespace py = pybind11;
using namespace gpumon;

namespace {

template <typename T>
void get(const py::dict& d, const char* k, T* out) {
  if (d.contains(k) && !d[k].is_none()) *out = d[k].cast<T>();
}

OnDeviceConfig ondevice_from(const py::dict& d) {
  OnDeviceConfig c;
  get(d, "plugin_dir", &c.plugin_dir);
  get(d, "pmc", &c.pmc);
  get(d, "pmc_counters", &c.pmc_counters);
  get(d, "pmc_every_s", &c.pmc_every_s);
  get(d, "pmc_window_s", &c.pmc_window_s);
  get(d, "pmc_mode", &c.pmc_mode);
  get(d, "ondevice_isolate", &c.ondevice_isolate);
  get(d, "helper_retry_s", &c.helper_retry_s);
  get(d, "probe", &c.probe);
  get(d, "probe_every_s", &c.probe_every_s);
  get(d, "probe_blocks", &c.probe_blocks);
  get(d, "probe_spin_ticks", &c.probe_spin_ticks);
  get(d, "probe_timeout_s", &c.probe_timeout_s);
  return c;
}

MockProc mock_proc_from(const py::dict& d) {
  MockProc p;
  get(d, "pid", &p.pid);
  get(d, "device", &p.device);
  get(d, "name", &p.name);
  get(d, "vram_bytes", &p.vram_bytes);
  get(d, "gfx_share", &p.gfx_share);
  get(d, "kfd_only", &p.kfd_only);
  get(d, "queues", &p.queues);
  return p;
}

ExporterConfig config_from(const py::dict& d) {
  ExporterConfig c;
  get(d, "backend", &c.backend);
  get(d, "amdsmi_lib", &c.amdsmi_lib);
  get(d, "rocm_smi_lib", &c.rocm_smi_lib);
  get(d, "fast_path", &c.fast_path);
  get(d, "sysfs_root", &c.sysfs_root);
  if (d.contains("devices") && !d["devices"].is_none())  // hip ids (int or str) and / or PCI BDFs
    for (auto x : d["devices"]) c.devices.push_back(py::str(x).cast<std::string>());
  get(d, "interval_s", &c.interval_s);
  get(d, "serve_http", &c.serve_http);
  get(d, "listen_addr", &c.listen_addr);
  get(d, "port", &c.port);
  get(d, "http_threads", &c.http_threads);
  get(d, "http_rt_priority", &c.http_rt_priority);
  get(d, "http_rt_budget", &c.http_rt_budget);
  get(d, "host", &c.host);
  get(d, "gzip", &c.gzip);
  get(d, "roctx", &c.roctx);
  get(d, "compat_families", &c.compat_families);
  get(d, "extended_families", &c.extended_families);
  get(d, "full_device_labels", &c.full_device_labels);
  get(d, "metrics_include", &c.metrics_include);
  get(d, "metrics_exclude", &c.metrics_exclude);
  get(d, "processes", &c.processes);
  get(d, "link_every", &c.link_every);
  get(d, "ras_every", &c.ras_every);
  get(d, "ras_slices", &c.ras_slices);
  get(d, "ras_async", &c.ras_async);
  get(d, "occ_samples", &c.occ_samples);
  get(d, "prewarm_ms", &c.prewarm_ms);
  get(d, "stale_hold_s", &c.stale_hold_s);
  get(d, "hide_empty_contexts", &c.hide_empty_contexts);
  get(d, "mfma_exclusive_window_s", &c.mfma_exclusive_window_s);
  get(d, "peer_context_max_vram_mib", &c.peer_context_max_vram_mib);
  get(d, "sample_threads", &c.sample_threads);
  get(d, "rt_priority", &c.rt_priority);
  get(d, "influx_url", &c.influx_url);
  get(d, "influx_extended", &c.influx_extended);
  get(d, "influx_gzip", &c.influx_gzip);
  get(d, "influx_schema", &c.influx_schema);
  get(d, "influx_every", &c.influx_every);
  get(d, "influx_timeout_s", &c.influx_timeout_s);
  get(d, "influx_token", &c.influx_token);
  get(d, "influx_ca_file", &c.influx_ca_file);
  get(d, "influx_tls_insecure", &c.influx_tls_insecure);
  get(d, "influx_client_cert", &c.influx_client_cert);
  get(d, "influx_client_key", &c.influx_client_key);
  get(d, "tls_cert_file", &c.tls_cert_file);
  get(d, "tls_key_file", &c.tls_key_file);
  get(d, "tls_client_ca_file", &c.tls_client_ca_file);
  get(d, "http_auth_token_file", &c.http_auth_token_file);
  get(d, "debug_listen", &c.debug_listen);
  get(d, "init_retry_s", &c.init_retry_s);
  get(d, "health_stale_s", &c.health_stale_s);
  get(d, "reinit_after", &c.reinit_after);
  get(d, "device_timeout_s", &c.device_timeout_s);
  get(d, "pod_resources_socket", &c.pod_resources_socket);
  get(d, "pod_resources_prefix", &c.pod_resources_prefix);
  get(d, "pod_resources_dra_drivers", &c.pod_resources_dra_drivers);
  get(d, "pod_resources_refresh_s", &c.pod_resources_refresh_s);
  get(d, "cri_socket", &c.cri_socket);
  get(d, "docker_socket", &c.docker_socket);
  get(d, "pod_log_root", &c.pod_log_root);
  get(d, "device_checkpoint", &c.device_checkpoint);
  get(d, "version", &c.version);
  get(d, "activity_acc_scale", &c.rates.activity_acc_scale);
  get(d, "xgmi_kb_bytes", &c.rates.xgmi_kb_bytes);
  get(d, "pcie_bw_unit_bytes", &c.rates.pcie_bw_unit_bytes);
  auto& a = c.attribution;
  get(d, "procfs_root", &a.procfs_root);
  get(d, "opt_in", &a.opt_in);
  get(d, "user_label", &a.user_label);
  get(d, "user_regex", &a.user_regex);
  get(d, "user_prefix", &a.user_prefix);
  get(d, "compat_user_rule", &a.compat_user_rule);
  get(d, "procfs_env_fallback", &a.procfs_env_fallback);
  get(d, "include_host_processes", &a.include_host_processes);
  get(d, "verify_kfd", &a.verify_kfd);
  get(d, "label_allowlist", &a.label_allowlist);
  if (d.contains("mock") && !d["mock"].is_none()) {
    py::dict m = d["mock"].cast<py::dict>();
    get(m, "gpus", &c.mock.gpus);
    get(m, "seed", &c.mock.seed);
    get(m, "mode", &c.mock.mode);
    get(m, "const_util", &c.mock.const_util);
    get(m, "hang_ms", &c.mock.hang_ms);
    get(m, "fail_device", &c.mock.fail_device);
    get(m, "fail_every", &c.mock.fail_every);
    get(m, "unsupported", &c.mock.unsupported);
    get(m, "n_xcd", &c.mock.n_xcd);
    get(m, "n_links", &c.mock.n_links);
    get(m, "firmware_hz", &c.mock.firmware_hz);
    if (m.contains("procs"))
      for (auto p : m["procs"].cast<py::list>()) c.mock.procs.push_back(mock_proc_from(p.cast<py::dict>()));
  }
  return c;
}

py::object num(double v) { return has(v) ? py::object(py::float_(v)) : py::object(py::none()); }

py::dict static_to_dict(const DeviceStatic& s) {
  py::dict d;
  d["index"] = s.index;
  d["hip_id"] = s.hip_id;
  d["gpu_id"] = s.gpu_id;
  d["uuid"] = s.uuid;
  d["bdf"] = s.bdf;
  d["model"] = s.model;
  d["serial"] = s.serial;
  d["gfx_target"] = s.gfx_target;
  d["compute_partition"] = s.compute_partition;
  d["memory_partition"] = s.memory_partition;
  d["drm_card"] = s.drm_card;
  d["drm_render"] = s.drm_render;
  d["kfd_node"] = s.kfd_node;
  d["partition_id"] = s.partition_id;
  d["num_cu"] = s.num_cu;
  d["driver_version"] = s.driver_version;
  d["driver_source"] = s.driver_source;
  d["vram_total_bytes"] = num(s.vram_total_bytes);
  d["power_limit_w"] = num(s.power_limit_w);
  return d;
}

py::dict sample_to_dict(const DeviceSample& s) {
  py::dict d;
  d["ok"] = s.ok;
  d["fresh"] = s.fresh;
  d["sample_ns"] = s.sample_ns;
  d["errors"] = s.errors;
  d["last_error"] = s.last_error;
  py::dict f;
  for (int i = 0; i < F_COUNT; ++i) f[field_name(i)] = num(s.v[i]);
  d["fields"] = f;
  py::list xb, gc, ht;
  for (int k = 0; k < s.n_xcd; ++k) xb.append(num(s.xcd_busy[k]));
  for (int k = 0; k < kMaxGfxClks; ++k) gc.append(num(s.gfxclks[k]));
  for (int k = 0; k < kMaxHbm; ++k) ht.append(num(s.hbm_temp[k]));
  d["xcd_busy"] = xb;
  d["gfxclks"] = gc;
  d["hbm_temp"] = ht;
  py::list links;
  for (int k = 0; k < s.n_links; ++k) {
    py::dict l;
    l["peer_bdf"] = s.links[k].peer_bdf;
    l["status"] = s.links[k].status;
    l["bit_rate_gbps"] = num(s.links[k].bit_rate_gbps);
    l["max_bandwidth_gbps"] = num(s.links[k].max_bandwidth_gbps);
    l["read_kb"] = s.acc.xgmi_rd_kb[k];
    l["write_kb"] = s.acc.xgmi_wr_kb[k];
    links.append(l);
  }
  d["links"] = links;
  if (s.ras.valid) {
    py::dict r;
    r["source"] = s.ras.source;
    py::dict blocks;
    for (const auto& c : s.ras.blocks) {
      py::dict b;
      b["ue"] = c.ue;
      b["ce"] = c.ce;
      if (c.has_de) b["de"] = c.de;
      blocks[py::str(c.block)] = b;
    }
    r["blocks"] = blocks;
    r["fatal"] = num(s.ras.fatal);
    r["poison_created"] = num(s.ras.poison_created);
    r["poison_consumed"] = num(s.ras.poison_consumed);
    r["bad_pages"] = num(s.ras.bad_pages);
    d["ras"] = r;
  } else {
    d["ras"] = py::none();
  }
  py::dict a;
  a["energy"] = s.acc.energy;
  a["accumulation_counter"] = s.acc.accumulation_counter;
  a["gfx_activity_acc"] = s.acc.gfx_activity_acc;
  a["mem_activity_acc"] = s.acc.mem_activity_acc;
  a["firmware_ts"] = s.acc.firmware_ts;
  a["system_clock_ns"] = s.acc.system_clock_ns;
  a["ppt_res"] = s.acc.ppt_res;
  a["pcie_bw_acc"] = s.acc.has_pcie_bw_acc ? py::object(py::int_(s.acc.pcie_bw_acc)) : py::object(py::none());
  py::list xa;
  for (int k = 0; k < s.acc.n_xcd_acc; ++k) xa.append(s.acc.xcd_busy_acc[k]);
  a["xcd_busy_acc"] = xa;
  d["acc"] = a;
  return d;
}

py::dict rates_to_dict(const DeviceRates& r) {
  py::dict d;
  d["valid"] = r.valid;
  d["dt_s"] = r.dt_s;
  d["power_from_energy_w"] = num(r.power_from_energy_w);
  d["ppt_violation_pct"] = num(r.ppt_violation_pct);
  d["thermal_violation_pct"] = num(r.thermal_violation_pct);
  d["gfx_activity_avg_pct"] = num(r.gfx_activity_avg_pct);
  d["mem_activity_avg_pct"] = num(r.mem_activity_avg_pct);
  py::list xb, rd, wr;
  for (int k = 0; k < r.n_xcd; ++k) xb.append(num(r.xcd_busy_avg[k]));
  for (int k = 0; k < r.n_links; ++k) {
    rd.append(num(r.xgmi_rd_Bps[k]));
    wr.append(num(r.xgmi_wr_Bps[k]));
  }
  d["xcd_busy_avg"] = xb;
  if (r.has_xcd_limit) {
    py::list lp, lt, la, lu;
    for (int k = 0; k < r.n_xcd; ++k) {
      lp.append(num(r.xcd_below_ppt_pct[k]));
      lt.append(num(r.xcd_below_thm_pct[k]));
      la.append(num(r.xcd_below_total_pct[k]));
      lu.append(num(r.xcd_low_util_pct[k]));
    }
    d["xcd_below_ppt_pct"] = lp;
    d["xcd_below_thm_pct"] = lt;
    d["xcd_below_total_pct"] = la;
    d["xcd_low_util_pct"] = lu;
  }
  d["xgmi_rd_Bps"] = rd;
  d["xgmi_wr_Bps"] = wr;
  d["pcie_Bps"] = num(r.pcie_Bps);
  return d;
}

py::dict row_to_dict(const PodRow& r) {
  py::dict d;
  d["dev"] = r.dev;
  d["idle"] = r.idle;
  d["pid"] = r.pid;
  d["procname"] = r.procname;
  d["namespace"] = r.pod_namespace;
  d["podname"] = r.pod_name;
  d["container"] = r.container;
  d["containerid"] = r.containerid;
  d["user_name"] = r.user_name;
  d["used_memory_bytes"] = r.used_memory_bytes;
  d["gpu_util"] = r.gpu_util;
  d["proc_gfx_util"] = num(r.proc_gfx_util);
  d["cu_occupancy"] = num(r.cu_occupancy);
  d["occ_samples"] = r.occ_samples;
  d["queues"] = r.queues;
  d["mfma_util"] = num(r.mfma_util);
  return d;
}

std::map<std::string, std::string> str_map(const py::dict& d, const char* k) {
  std::map<std::string, std::string> m;
  if (d.contains(k) && !d[k].is_none())
    for (auto kv : d[k].cast<py::dict>()) m[kv.first.cast<std::string>()] = kv.second.cast<std::string>();
  return m;
}

MockBackend* mock_of(Exporter& e) {
  auto* m = dynamic_cast<MockBackend*>(e.backend());
  if (!m) throw std::runtime_error("exporter backend is not the mock backend");
  return m;
}

// A Python value as the option setters take it: strings, one per list element; bools as true/false.
std::vector<std::string> option_values(py::handle v) {
  auto one = [](py::handle x) -> std::string {
    if (py::isinstance<py::bool_>(x)) return x.cast<bool>() ? "true" : "false";
    return py::str(x).cast<std::string>();
  };
  std::vector<std::string> out;
  if (v.is_none()) return out;
  if (py::isinstance<py::list>(v) || py::isinstance<py::tuple>(v)) {
    for (auto x : v) out.push_back(one(x));
    if (out.empty()) out.push_back("");  // [] -> an empty list key / an empty string
    return out.size() == 1 && out[0].empty() ? std::vector<std::string>{} : out;
  }
  out.push_back(one(v));
  return out;
}

std::vector<std::string> env_strings(const py::dict& env) {
  std::vector<std::string> kv;
  for (auto item : env) kv.push_back(py::str(item.first).cast<std::string>() + "=" + py::str(item.second).cast<std::string>());
  return kv;
}

struct EnvBlock {  // char** view of "k=v" strings
  explicit EnvBlock(std::vector<std::string> kv) : s(std::move(kv)) {
    for (auto& x : s) p.push_back(x.data());
    p.push_back(nullptr);
  }
  std::vector<std::string> s;
  std::vector<char*> p;
};

}  // namespace

static py::dict tick_to_dict(const TickInfo& t) {
  py::dict d;
  d["seq"] = t.seq;
  d["duration_s"] = t.duration_s;
  d["devices"] = t.devices;
  d["devices_ok"] = t.devices_ok;
  d["pod_rows"] = t.pod_rows;
  d["body_bytes"] = t.body_bytes;
  d["t_sample"] = t.t_sample;
  d["t_procs"] = t.t_procs;
  d["t_attrib"] = t.t_attrib;
  d["t_render"] = t.t_render;
  d["t_gzip"] = t.t_gzip;
  d["t_wake"] = t.t_wake;
  d["t_device"] = t.t_device;
  d["t_late"] = t.t_late;
  d["link_refreshes"] = t.link_refreshes;
  d["ras_reads"] = t.ras_reads;
  d["ras_full"] = t.ras_full;
  py::list dev;
  for (const auto& x : t.dev) {
    py::dict e;
    e["ok"] = x.ok;
    e["fresh"] = x.fresh;
    e["rates_valid"] = x.rates_valid;
    e["gfx_util"] = num(x.gfx_util);
    e["xgmi_wr_Bps"] = num(x.xgmi_wr_Bps);
    e["xgmi_rd_Bps"] = num(x.xgmi_rd_Bps);
    e["pcie_Bps"] = num(x.pcie_Bps);
    e["t_device"] = x.t_device;
    e["t_procs"] = x.t_procs;
    dev.append(e);
  }
  d["dev"] = dev;
  return d;
}

PYBIND11_MODULE(_core, m) {
  m.doc() = "gpumon C++ core (MI355X telemetry exporter)";

  m.def("set_log_level", [](int lvl) { g_log_level.store(lvl); });
  m.def("glob_match", [](const std::string& glob, const std::string& name) { return glob_match(glob.c_str(), name.c_str()); },
        py::arg("glob"), py::arg("name"), "the family-filter glob rule (render.h)");
  m.def("parse_cgroup", [](const std::string& text) {
    CgroupInfo c = parse_cgroup(text);
    py::dict d;
    d["found"] = c.found;
    d["runtime"] = c.runtime;
    d["container_id"] = c.container_id;
    d["pod_uid"] = c.pod_uid;
    d["qos"] = c.qos;
    return d;
  });
  m.def("compat_user_from_pod", &compat_user_from_pod, py::arg("pod_name"),
        py::arg("prefix") = "turing-gpu-notebook-");
  m.def("escape_label_value", [](const std::string& s) {
    std::string o;
    escape_label_value(s, &o);
    return o;
  });
  m.def("escape_influx_tag", [](const std::string& s) {
    std::string o;
    escape_influx_tag(s, &o);
    return o;
  });
  m.def("escape_influx_field_str", [](const std::string& s) {
    std::string o;
    escape_influx_field_str(s, &o);
    return o;
  });
  m.def("format_double", [](double v) {
    std::string o;
    append_double(v, &o);
    return o;
  });
  m.def(
      "amdsmi_compare_tables",
      [](const std::string& lib, const std::string& sys_root, int dev) {
        AmdSmiBackend b(lib);
        b.set_fast_path(true, sys_root, "/proc");
        std::string err;
        py::dict r;
        if (!b.init(&err)) {
          r["error"] = err;
          return r;
        }
        r["fast_path_devices"] = b.fast_path_devices();
        r["fast_path_status"] = b.fast_path_status();
        py::list rows;
        for (const auto& [name, a, s] : b.compare_tables(dev, &err)) rows.append(py::make_tuple(name, a, s));
        r["rows"] = rows;
        r["error"] = err;
        return r;
      },
      py::arg("lib") = "", py::arg("sys_root") = "/sys", py::arg("dev") = 0,
      "libamd_smi vs sysfs-decoded gpu_metrics v1.8, field by field: (name, amdsmi, sysfs)");
  m.def(
      "podresources_list",
      [](const std::string& sock, const std::string& prefix, int timeout_ms, const std::vector<std::string>& dra) {
        std::vector<PodDeviceRow> rows;
        std::string err;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = podresources_list(sock, prefix, &rows, &err, timeout_ms, dra);
        }
        if (!ok) throw std::runtime_error(err);
        py::list l;
        for (const auto& r : rows) {
          py::dict d;
          d["namespace"] = r.pod_namespace;
          d["pod"] = r.pod_name;
          d["container"] = r.container_name;
          d["resource"] = r.resource_name;
          d["device_id"] = r.device_id;
          l.append(d);
        }
        return l;
      },
      py::arg("socket"), py::arg("resource_prefix") = "amd.com/gpu", py::arg("timeout_ms") = 3000,
      py::arg("dra_drivers") = std::vector<std::string>{"gpu.amd.com"},
      "kubelet PodResources List() through the native HTTP/2 client (grpc_lite.cpp)");
  m.def(
      "grpc_call",
      [](const std::string& sock, const std::string& path, py::bytes req, int timeout_ms) {
        std::string resp, err;
        GrpcStatus st;
        bool ok;
        const std::string r = req;
        {
          py::gil_scoped_release nogil;
          ok = grpc_unary_unix(sock, path, r, &resp, &err, timeout_ms, &st);
        }
        py::dict d;
        d["ok"] = ok;
        d["response"] = py::bytes(resp);
        d["error"] = err;
        d["code"] = st.code;
        d["code_name"] = st.code >= 0 ? std::string(grpc_code_name(st.code)) : std::string();
        d["message"] = st.message;
        d["http_status"] = st.http_status;
        return d;
      },
      py::arg("socket"), py::arg("path"), py::arg("request") = py::bytes(""), py::arg("timeout_ms") = 3000,
      "one unary call through grpc_lite.cpp with the server's decoded status");
  m.def(
      "hpack_decode",
      [](const std::vector<py::bytes>& blocks, size_t table_size) {
        HpackDecoder dec(table_size);
        py::list out;
        for (const auto& b : blocks) {
          HeaderList h;
          std::string err;
          if (!dec.decode(std::string(b), &h, &err)) throw py::value_error(err);
          py::list l;
          for (const auto& [k, v] : h) l.append(py::make_tuple(k, v));
          py::dict d;
          d["headers"] = l;
          d["table_size"] = dec.table_size();
          d["table_entries"] = dec.table_entries();
          out.append(d);
        }
        return out;
      },
      py::arg("blocks"), py::arg("table_size") = 4096,
      "decode consecutive HPACK header blocks of one connection (hpack.cpp)");
  m.def("hpack_huffman_encode", [](py::bytes s) { return py::bytes(hpack_huffman_encode(std::string(s))); });
  m.def("hpack_huffman_decode", [](py::bytes b) {
    std::string out;
    if (!hpack_huffman_decode(std::string(b), &out)) throw py::value_error("invalid Huffman string");
    return py::bytes(out);
  });
  auto docker_rows = [](const std::vector<DockerContainer>& cs) {
    py::list l;
    for (const auto& c : cs) {
      py::dict d;
      d["id"] = c.id;
      d["name"] = c.name;
      d["state"] = c.state;
      d["labels"] = c.labels;
      l.append(d);
    }
    return l;
  };
  m.def(
      "docker_parse_containers",
      [docker_rows](py::bytes b) {
        std::vector<DockerContainer> cs;
        std::string err;
        if (!docker_parse_containers(std::string(b), &cs, &err)) throw py::value_error(err);
        return docker_rows(cs);
      },
      py::arg("json"), "parse a Docker Engine GET /containers/json body (docker_lite.cpp)");
  m.def(
      "device_checkpoint_parse",
      [](py::bytes b) {
        std::vector<CheckpointEntry> es;
        std::string err;
        if (!device_checkpoint_parse(std::string(b), &es, &err)) throw py::value_error(err);
        py::list out;
        for (const auto& e : es) {
          py::dict d;
          d["pod_uid"] = py::bytes(e.pod_uid);
          d["container"] = py::bytes(e.container_name);
          d["resource"] = py::bytes(e.resource);
          py::list ids;
          for (const auto& x : e.device_ids) ids.append(py::bytes(x));
          d["device_ids"] = ids;
          out.append(d);
        }
        return out;
      },
      py::arg("json"), "parse the kubelet device-plugin checkpoint (kubelet_files.cpp)");
  m.def(
      "container_log_name",
      [](const std::string& name) -> py::object {
        std::string pod, ns, ctr, id;
        if (!parse_container_log_name(name, &pod, &ns, &ctr, &id)) return py::none();
        return py::make_tuple(pod, ns, ctr, id);
      },
      py::arg("name"), "split /var/log/containers/<pod>_<ns>_<container>-<id>.log (kubelet_files.cpp)");
  m.def(
      "http1_parse_response",
      [](py::bytes raw, bool eof) {
        int status = -1;
        std::string body, err;
        if (!http1_parse_response(std::string(raw), &status, &body, &err, eof)) throw py::value_error(err);
        return py::make_tuple(status, py::bytes(body));
      },
      py::arg("raw"), py::arg("eof") = true);
  m.def(
      "docker_list",
      [docker_rows](const std::string& sock, int timeout_ms) {
        std::vector<DockerContainer> cs;
        std::string err;
        int status = -1;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = docker_list(sock, &cs, &err, timeout_ms, &status);
        }
        if (!ok) throw std::runtime_error(err);
        return docker_rows(cs);
      },
      py::arg("socket"), py::arg("timeout_ms") = 3000, "Docker Engine GET /containers/json via docker_lite.cpp");
  m.def(
      "parse_cri_containers",
      [](py::bytes msg) {
        std::vector<CriContainer> cs;
        if (!parse_cri_containers(std::string(msg), &cs)) throw std::runtime_error("malformed ListContainersResponse");
        py::list out;
        for (const auto& c : cs)
          out.append(py::make_tuple(c.id, c.sandbox_id, c.name, c.labels, c.annotations));
        return out;
      },
      "runtime.v1 ListContainersResponse -> [(id, sandbox_id, name, labels, annotations)] (grpc_lite.cpp)");
  m.def(
      "parse_cri_sandboxes",
      [](py::bytes msg) {
        std::vector<CriSandbox> ss;
        if (!parse_cri_sandboxes(std::string(msg), &ss)) throw std::runtime_error("malformed ListPodSandboxResponse");
        py::list out;
        for (const auto& s : ss)
          out.append(py::make_tuple(s.id, s.name, s.uid, s.pod_namespace, s.labels, s.annotations));
        return out;
      },
      "runtime.v1 ListPodSandboxResponse -> [(id, name, uid, namespace, labels, annotations)] (grpc_lite.cpp)");
  m.def(
      "cri_list",
      [](const std::string& sock, int timeout_ms) {
        std::vector<CriContainer> cs;
        std::vector<CriSandbox> sbs;
        std::string err;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = cri_list(sock, &cs, &sbs, &err, timeout_ms);
        }
        if (!ok) throw std::runtime_error(err);
        py::list lc, ls;
        for (const auto& c : cs) {
          py::dict d;
          d["id"] = c.id;
          d["sandbox_id"] = c.sandbox_id;
          d["name"] = c.name;
          d["labels"] = c.labels;
          d["annotations"] = c.annotations;
          lc.append(d);
        }
        for (const auto& s : sbs) {
          py::dict d;
          d["id"] = s.id;
          d["name"] = s.name;
          d["uid"] = s.uid;
          d["namespace"] = s.pod_namespace;
          d["labels"] = s.labels;
          d["annotations"] = s.annotations;
          ls.append(d);
        }
        return py::make_tuple(lc, ls);
      },
      py::arg("socket"), py::arg("timeout_ms") = 3000, "CRI ListContainers + ListPodSandbox via grpc_lite.cpp");
  m.def(
      "parse_list_pod_resources",
      [](py::bytes b, const std::string& prefix, const std::vector<std::string>& dra) {
        std::vector<PodDeviceRow> rows;
        std::string s = b;
        if (!parse_list_pod_resources(s, prefix, &rows, dra)) throw std::runtime_error("malformed");
        py::list l;
        for (const auto& r : rows)
          l.append(py::make_tuple(r.pod_namespace, r.pod_name, r.container_name, r.resource_name, r.device_id));
        return l;
      },
      py::arg("data"), py::arg("resource_prefix") = "", py::arg("dra_drivers") = std::vector<std::string>{});
  m.def(
      "match_device_id",
      [](const std::string& id, const py::list& statics) {
        std::vector<DeviceStatic> st;
        for (auto o : statics) {
          py::dict d = o.cast<py::dict>();
          DeviceStatic s;
          get(d, "index", &s.index);
          get(d, "hip_id", &s.hip_id);
          get(d, "bdf", &s.bdf);
          get(d, "uuid", &s.uuid);
          get(d, "drm_card", &s.drm_card);
          get(d, "drm_render", &s.drm_render);
          st.push_back(s);
        }
        return match_device_id(id, st);
      },
      "C++ twin of tests/oracles/attribution/plane.py match_device_id (the native PodResources poller's matcher)");
  m.def(
      "docker_parse_inspect",
      [](py::bytes b) {
        DockerInspect di;
        std::string err;
        if (!docker_parse_inspect(std::string(b), &di, &err)) throw py::value_error(err);
        py::dict d;
        d["id"] = di.id;
        d["devices"] = di.devices;
        d["env"] = di.env;
        return d;
      },
      py::arg("json"));
  m.def(
      "docker_container_gpus",
      [](const std::vector<std::string>& devices, const std::vector<std::string>& env, const py::list& statics) {
        std::vector<DeviceStatic> st;
        for (auto o : statics) {
          py::dict d = o.cast<py::dict>();
          DeviceStatic s;
          get(d, "index", &s.index);
          get(d, "hip_id", &s.hip_id);
          get(d, "bdf", &s.bdf);
          get(d, "uuid", &s.uuid);
          get(d, "drm_card", &s.drm_card);
          get(d, "drm_render", &s.drm_render);
          st.push_back(s);
        }
        DockerInspect di;
        di.devices = devices;
        di.env = env;
        return Exporter::docker_container_gpus(di, st);
      },
      py::arg("devices"), py::arg("env"), py::arg("statics"));
  m.def("roctx_enable", &Roctx::enable, py::arg("on") = true,
        "Load librocprofiler-sdk-roctx and bracket sampler phases with ROCTx ranges");
  m.def("roctx_active", &Roctx::active);
  m.def("roctx_ranges", &Roctx::ranges, "ROCTx ranges opened so far by this process");
  m.def(
      "fd_table_stats",
      [] {
        py::dict d;
        d["scans"] = gpumon::DrmFdTables::get().scans();
        d["entries"] = gpumon::DrmFdTables::get().size();
        return d;
      },
      "node-wide /proc/<pid>/fd scan cache of the sysfs fast path (scans so far, cached processes)");
  m.def("fd_table_scans_of", [](const std::string& pdir) { return gpumon::DrmFdTables::get().scans_of(pdir); },
        py::arg("pdir"), "scans of one /proc/<pid> entry of the fd-table cache (0 when not cached)");
  m.def("fd_table_clear", [] { gpumon::DrmFdTables::get().clear(); },
        "drop every cached fd table (tests: entries of an earlier test's fake /proc tree)");
  m.def("gzip", [](const std::string& s) {
    std::string o;
    if (!gzip_compress(s, &o)) throw std::runtime_error("gzip failed");
    return py::bytes(o);
  });
  m.def(
      "snapshot_gzip_race",
      [](const std::string& body, int threads, bool during_precompress) {
        // `threads` scrapes ask one fresh snapshot for gzip at the same instant -- or, with
        // during_precompress, while the tick thread's precompress() of it is running. Exactly one
        // thread compresses; the others wait for it, at most Snapshot::kGzipWaitNs. Returns (the
        // gzip body every thread got, or None if any got none; distinct buffers handed out, 1 =
        // compressed once; scrapes that started while the compression was in flight; the longest
        // any scrape thread spent in gzipped(), seconds -- for a waiter, how long its loop stalled).
        auto snap = std::make_shared<gpumon::Snapshot>();
        snap->body = body;
        snap->gzip = true;
        std::vector<const std::string*> got(std::max(threads, 1), nullptr);
        std::vector<double> spent(got.size(), 0.0);
        std::atomic<int> mid{0};
        {
          py::gil_scoped_release nogil;
          std::thread pre;
          if (during_precompress) {
            pre = std::thread([&] { (void)snap->precompress(); });
            while (!snap->compressing() && !snap->compressed()) std::this_thread::yield();
          }
          std::atomic<int> ready{0};
          std::vector<std::thread> th;
          for (size_t i = 0; i < got.size(); ++i)
            th.emplace_back([&, i] {
              ready.fetch_add(1);
              while (ready.load() < static_cast<int>(got.size())) std::this_thread::yield();
              const bool waiter = snap->compressing();
              if (waiter) mid.fetch_add(1);
              const int64_t t0 = gpumon::mono_ns();
              got[i] = snap->gzipped(true);
              if (waiter) spent[i] = (gpumon::mono_ns() - t0) * 1e-9;
            });
          for (auto& t : th) t.join();
          if (pre.joinable()) pre.join();
        }
        std::set<const std::string*> distinct(got.begin(), got.end());
        const bool all = std::find(got.begin(), got.end(), nullptr) == got.end();
        return py::make_tuple(all ? py::object(py::bytes(*got[0])) : py::object(py::none()),
                              static_cast<int>(distinct.size()), mid.load(),
                              *std::max_element(spent.begin(), spent.end()));
      },
      py::arg("body"), py::arg("threads") = 8, py::arg("during_precompress") = false);
  m.def(
      "scrape_load",
      [](const std::string& host, int port, const std::string& path, int n, double duration_s,
         int concurrency, double rate_hz, bool keep_alive, bool gzip) {
        ScrapeStats s;
        {
          py::gil_scoped_release nogil;
          s = scrape_load(host, port, path, n, duration_s, concurrency, rate_hz, keep_alive, gzip);
        }
        py::dict d;
        d["latencies_s"] = s.latencies_s;
        d["errors"] = s.errors;
        d["bytes"] = s.bytes;
        d["wall_s"] = s.wall_s;
        return d;
      },
      py::arg("host"), py::arg("port"), py::arg("path") = "/metrics", py::arg("n_requests") = 100,
      py::arg("duration_s") = 0.0, py::arg("concurrency") = 1, py::arg("rate_hz") = 0.0,
      py::arg("keep_alive") = true, py::arg("gzip") = false);
  m.def("parse_url", [](const std::string& url) {
    const Url u = parse_url(url);
    py::dict d;
    d["ok"] = u.ok;
    d["host"] = u.host;
    d["port"] = u.port;
    d["path"] = u.path;
    d["auth_header"] = u.auth_header;
    d["tls"] = u.tls;
    d["error"] = u.error;
    return d;
  });
  // Configuration-time check shared by both entry points: "" = usable push config, else the reason.
  m.def(
      "check_push_config",
      [](const std::string& url, const std::string& token, const std::string& ca_file, bool insecure,
         const std::string& client_cert, const std::string& client_key) {
        TlsOptions t;
        t.ca_file = ca_file;
        t.insecure = insecure;
        t.client_cert = client_cert;
        t.client_key = client_key;
        return check_push_config(url, token, t);
      },
      py::arg("url"), py::arg("token") = "", py::arg("ca_file") = "", py::arg("insecure") = false,
      py::arg("client_cert") = "", py::arg("client_key") = "");
  m.def(
      "serve_tls_not_after",
      [](const std::string& cert, const std::string& key, const std::string& ca) {
        // (error, expiry of the serving certificate in unix seconds): the doctor's TLS check
        std::string err;
        auto t = TlsServer::create(cert, key, ca, &err);
        return py::make_tuple(err, t ? t->not_after() : 0);
      },
      py::arg("cert_file"), py::arg("key_file"), py::arg("client_ca_file") = "");
  m.def(
      "read_token_file",
      [](const std::string& path) {
        std::vector<std::string> toks;
        std::string err = read_token_file(path, &toks);
        return py::make_tuple(err, toks.empty() ? std::string() : toks.front(), toks);
      },
      py::arg("path"), "(error, first token, all tokens): the token file format http_auth_token_file reads");
  m.def("check_auth_token_file", &check_auth_token_file, py::arg("path") = "",
        "'' when the bearer-token file for /metrics is unset or holds a usable token, else the reason");
  m.def("check_serve_tls", &check_serve_tls, py::arg("cert_file") = "", py::arg("key_file") = "",
        py::arg("client_ca_file") = "", "configuration-time check of the /metrics HTTPS files: \"\" = usable");
  m.def("redact_url", &redact_url);
  m.def("driver_version_label", [](const std::string& raw, const std::string& module_version) {
    std::string source;
    std::string v = driver_version_label(raw, module_version, &source);
    return py::make_tuple(v, source);
  }, py::arg("raw"), py::arg("module_version") = "",
     "gpu_info driver_version label and its source (module | kernel | library) from libamd_smi's string");
  m.def("parse_listen", [](const std::string& l) {
    std::string host, err;
    int port = -1;
    const bool ok = parse_listen(l, &host, &port, &err);
    return py::make_tuple(ok, host, port, err);
  });
  m.def(
      "http_request",
      [](const std::string& method, const std::string& url, const std::string& body,
         const std::string& headers, double timeout_s, const std::string& ca_file, bool insecure, int repeat) {
        HttpClient c(timeout_s);
        std::string resp, err;
        int st = -1;
        {
          py::gil_scoped_release nogil;
          const Url u = parse_url(url);
          if (!u.ok) {
            err = u.error;
          } else {
            if (u.tls) {
              TlsOptions t;
              t.ca_file = ca_file;
              t.insecure = insecure;
              auto ctx = TlsContext::create(t, &err);
              if (ctx) c.set_tls(std::move(ctx));
            }
            // `repeat` requests over the one client (keep-alive reuse); the last result is returned
            if (err.empty())
              for (int i = 0; i < std::max(1, repeat); ++i) st = c.request(method, u, body, headers, &resp, &err);
          }
        }
        return py::make_tuple(st, py::bytes(resp), err);
      },
      py::arg("method"), py::arg("url"), py::arg("body") = "", py::arg("headers") = "",
      py::arg("timeout_s") = 5.0, py::arg("ca_file") = "", py::arg("insecure") = false, py::arg("repeat") = 1);

  // xGMI link-metrics entry -> gpu_metrics slot pairing (xgmi_map.h), for direct unit tests.
  py::class_<XgmiSlotMap>(m, "XgmiSlotMap")
      .def(py::init<>())
      .def(
          "update",
          [](XgmiSlotMap& mp, const py::list& entries, const std::vector<uint64_t>& rd, const std::vector<uint64_t>& wr,
             const std::vector<int>& status) {
            DeviceSample s;
            s.acc.valid = true;
            s.acc.n_links_acc = static_cast<int>(std::min<size_t>(rd.size(), kMaxLinks));
            for (int k = 0; k < s.acc.n_links_acc; ++k) {
              s.acc.xgmi_rd_kb[k] = rd[k];
              s.acc.xgmi_wr_kb[k] = k < static_cast<int>(wr.size()) ? wr[k] : 0;
              s.links[k].status = k < static_cast<int>(status.size()) ? status[k] : 1;
            }
            for (auto e : entries) {
              auto d = e.cast<py::dict>();
              LinkEntry le;
              le.peer_bdf = d.contains("bdf") ? d["bdf"].cast<std::string>() : "";
              le.read_kb = d.contains("read") ? d["read"].cast<uint64_t>() : 0;
              le.write_kb = d.contains("write") ? d["write"].cast<uint64_t>() : 0;
              le.has_acc = !d.contains("has_acc") || d["has_acc"].cast<bool>();
              s.link_entries.push_back(le);
            }
            mp.update(s);
            std::vector<int> slots;
            for (size_t j = 0; j < s.link_entries.size(); ++j) slots.push_back(mp.slot_of(j));
            return slots;
          },
          py::arg("entries"), py::arg("rd"), py::arg("wr"), py::arg("status"),
          "one link refresh: entries [{bdf, read, write}], the table slots' read / write KB and status; "
          "returns the slot paired with each entry (-1 = none)")
      .def_property_readonly("verified", &XgmiSlotMap::verified)
      .def_property_readonly("unverified", &XgmiSlotMap::unverified)
      .def_property_readonly("mismatched", &XgmiSlotMap::mismatched);

  // The one configuration implementation (csrc/core/options.h); gpumon/config.py is a view of it.
  py::class_<NativeOptions>(m, "Options")
      .def(py::init<>())
      .def("copy", [](const NativeOptions& o) { return NativeOptions(o); })
      .def("set",
           [](NativeOptions& o, const std::string& key, py::handle v) {
             std::string err;
             const int r = options_set(&o, key, option_values(v), &err);
             if (r == 0) throw py::key_error("unknown config key: " + key);
             if (r < 0) throw py::value_error(err);
           },
           py::arg("key"), py::arg("value"))
      .def("load_file",
           [](NativeOptions& o, const std::string& path) {
             std::vector<std::string> unknown;
             std::string err;
             if (!options_load_file(&o, path, &unknown, &err)) throw py::value_error(err);
             return unknown;
           },
           "apply a YAML config file; returns the keys it does not know (ignored)")
      .def("apply_env",
           [](NativeOptions& o, const py::dict& env) {
             EnvBlock e(env_strings(env));
             std::string err;
             std::vector<std::string> unknown;
             if (!options_apply_env(&o, e.p.data(), &err, &unknown)) throw py::value_error(err);
             return unknown;  // GPUMON_* names that are neither keys nor environment-only variables
           })
      .def_static(
          "parse",
          [](const std::vector<std::string>& args, const py::dict& env) {
            NativeOptions o;
            EnvBlock e(env_strings(env));
            std::vector<std::string> rest, warnings;
            std::string err;
            if (options_parse(&o, args, e.p.data(), &rest, &warnings, &err) != ParseStatus::kOk)
              throw py::value_error(err);
            return py::make_tuple(o, rest, warnings);
          },
          py::arg("args"), py::arg("env"),
          "file < environment < --compat < flags over a command line: (Options, other args, warnings)")
      .def("finalized",
           [](const NativeOptions& o) {
             NativeOptions c = o;
             std::string err;
             if (!options_finalize(&c, &err)) throw py::value_error(err);
             return c;
           },
           "a copy with the listen address, host fallback and control-plane sockets resolved")
      .def("validate", &options_validate, "'' or why the configuration cannot run (finalized options)")
      .def("to_json", [](const NativeOptions& o, bool redact) { return options_json(o, redact); },
           py::arg("redact") = false)
      .def_property_readonly("listen_addr", [](const NativeOptions& o) { return o.cfg.listen_addr; })
      .def_property_readonly("port", [](const NativeOptions& o) { return o.cfg.port; })
      .def_property_readonly("host", [](const NativeOptions& o) { return o.cfg.host; })
      .def_property_readonly("log_level_value", &options_log_level)
      .def_property_readonly("exporter_sources", [](const NativeOptions& o) {
        py::dict d;  // what a finalized configuration hands the exporter's pollers
        d["pod_resources_socket"] = o.cfg.pod_resources_socket;
        d["cri_socket"] = o.cfg.cri_socket;
        d["docker_socket"] = o.cfg.docker_socket;
        d["pod_log_root"] = o.cfg.pod_log_root;
        d["device_checkpoint"] = o.cfg.device_checkpoint;
        return d;
      });
  m.def("option_keys", [] {
    py::list l;
    for (const auto& k : option_keys()) {
      py::dict d;
      d["key"] = k.key;
      d["section"] = k.section;
      d["help"] = k.help;
      l.append(d);
    }
    return l;
  }, "every configuration key with its documentation section and help");
  m.def("option_flags", [] {
    py::list l;
    for (const auto& f : option_flags()) {
      py::dict d;
      d["flag"] = f.flag;
      py::list al;
      for (const auto& a : split(f.aliases, ','))
        if (!a.empty()) al.append(a);
      d["aliases"] = al;
      d["key"] = f.key;
      d["fixed"] = f.fixed ? py::object(py::str(f.fixed)) : py::object(py::none());
      d["help"] = f.help;
      l.append(d);
    }
    return l;
  }, "the command-line flags both entry points take");
  m.def("memory_limit_bytes", &memory_limit_bytes, py::arg("proc_cgroup") = "/proc/self/cgroup",
        py::arg("cgroup_root") = "/sys/fs/cgroup", "the memory limit the HTTP connection cap is sized against");
  m.def(
      "kfd_queue_scans",
      [](const std::string& sys_root, uint32_t pid) {
        return KfdQueueTables::get().scans_of(sys_root + "/class/kfd/kfd/proc", pid);
      },
      "scans of a process's KFD queue list so far (node-wide table shared by every GPU's worker)");
  m.def("kfd_queue_tables_clear", [] { KfdQueueTables::get().clear(); },
        "forget every cached KFD queue list (tests that rewrite a fake tree within the rescan period)");
  m.def("env_only_variables", &env_only_variables,
        "GPUMON_* variables read by the runtime that are not configuration keys (docs/configuration.md)");
  m.def("cri_autodetect_sockets", &cri_autodetect_sockets);

  py::class_<Exporter>(m, "Exporter")
      .def(py::init([](const NativeOptions& o) { return new Exporter(o.cfg); }),
           "from finalized Options (gpumon.config.Config.finalized())")
      .def(py::init([](const py::dict& cfg) { return new Exporter(config_from(cfg)); }))
      .def("start",
           [](Exporter& e) {
             std::string err;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = e.start(&err);
             }
             if (!ok) throw std::runtime_error("exporter start failed: " + err);
             return err;  // non-fatal backend error (retrying), or ""
           })
      .def("stop", [](Exporter& e) {
        py::gil_scoped_release nogil;
        e.stop();
      })
      .def("tick",
           [](Exporter& e) {
             TickInfo t;
             {
               py::gil_scoped_release nogil;
               t = e.tick();
             }
             return tick_to_dict(t);
           })
      .def("tick_log",
           [](const Exporter& e) {
             py::list l;
             for (const auto& t : e.tick_log()) l.append(tick_to_dict(t));
             return l;
           },
           "the last 4096 ticks (TickInfo dicts, oldest first): per-tick phase times for tail attribution")
      .def("phase_totals", &Exporter::phase_totals)
      .def("wait_for_seq",
           [](Exporter& e, uint64_t seq, double timeout_s) {
             py::gil_scoped_release nogil;
             return e.wait_for_seq(seq, timeout_s);
           })
      .def_property_readonly("port", &Exporter::port)
      .def_property_readonly("debug_port", &Exporter::debug_port)
      .def(
          "debug_view",
          [](Exporter& e, const std::string& path) {
            std::string body;
            {
              py::gil_scoped_release nogil;  // /debug/wait blocks until a tick
              body = e.debug_view(path);
            }
            if (body.empty()) throw py::key_error("no introspection view " + path);
            return py::module_::import("json").attr("loads")(body);
          },
          py::arg("path"), "an introspection view (/debug/state, /debug/procs, ...) as parsed JSON")
      .def_property_readonly("seq", &Exporter::seq)
      .def("healthy", &Exporter::healthy)
      .def("ready", &Exporter::ready)
      .def("metrics_text",
           [](Exporter& e) {
             auto s = e.snapshot();
             return s ? s->body : std::string();
           })
      .def("reload_tls", &Exporter::reload_tls, "re-check the /metrics TLS files now (SIGHUP)")
      .def("metrics_gzip",
           [](Exporter& e) {
             auto s = e.snapshot();
             const std::string* g = s ? s->gzipped(true) : nullptr;
             return py::bytes(g ? *g : std::string());
           })
      .def("influx_text", &Exporter::render_influx_now)
      .def_property_readonly("listen_desc", &Exporter::listen_desc)
      .def("statics",
           [](Exporter& e) {
             py::list l;
             for (const auto& s : e.statics()) l.append(static_to_dict(s));
             return l;
           })
      .def("samples",
           [](Exporter& e) {
             py::list l;
             for (const auto& s : e.samples()) l.append(sample_to_dict(s));
             return l;
           })
      .def("rates",
           [](Exporter& e) {
             py::list l;
             for (const auto& r : e.rates()) l.append(rates_to_dict(r));
             return l;
           })
      .def("pod_rows",
           [](Exporter& e) {
             py::list l;
             for (const auto& r : e.pod_rows()) l.append(row_to_dict(r));
             return l;
           })
      .def("self_stats",
           [](Exporter& e) {
             SelfStats s = e.self_stats();
             py::dict d;
             d["ticks"] = s.ticks;
             d["samples"] = s.samples;
             d["stale_samples"] = s.stale_samples;
             d["frozen_samples"] = s.frozen_samples;
             d["occupancy_reads"] = s.occupancy_reads;
             d["occupancy_scan_failures"] = s.occupancy_scan_failures;
             d["process_list_failures"] = s.process_list_failures;
             d["http_rt_loops"] = s.http_rt_loops;
             d["http_rt_demotions"] = s.http_rt_demotions;
             d["http_evicted"] = s.http_evicted;
             d["http_max_conns"] = s.http_max_conns;
             d["http_tls_failures"] = s.http_tls_failures;
             d["http_tls_client_cert_refused"] = s.http_tls_client_cert_refused;
             d["http_tls_not_after"] = s.http_tls_not_after;
             d["http_tls_reloads_ok"] = s.http_tls_reloads_ok;
             d["http_tls_reloads_failed"] = s.http_tls_reloads_failed;
             d["http_auth_failures"] = s.http_auth_failures;
             d["http_auth_reloads_ok"] = s.http_auth_reloads_ok;
             d["http_auth_reloads_failed"] = s.http_auth_reloads_failed;
             d["hidden_contexts"] = s.hidden_contexts;
             d["hidden_peer_contexts"] = s.hidden_peer_contexts;
             d["rt_threads"] = s.rt_threads;
             d["overruns"] = s.overruns;
             d["scrapes"] = s.scrapes;
             d["http_connections"] = s.http_connections;
             d["pods_attributed"] = s.pods_attributed;
             d["backend"] = s.backend;
             d["backend_version"] = s.backend_version;
             d["backend_up"] = s.backend_up;
             d["backend_reinits"] = s.backend_reinits;
             d["fast_path_devices"] = s.fast_path_devices;
             d["fast_path_status"] = s.fast_path_status;
             py::dict calls;
             for (const auto& c : s.backend_calls) {
               py::dict cd;
               cd["n"] = c.n;
               cd["errors"] = c.errors;
               cd["seconds"] = c.seconds;
               calls[py::str(c.call)] = cd;
             }
             d["backend_calls"] = calls;
             d["influx_ok"] = s.influx_ok;
             d["influx_fail"] = s.influx_fail;
             d["influx_dropped"] = s.influx_dropped;
             d["influx_enabled"] = s.influx_enabled;
             d["influx_up"] = s.influx_up;
             d["gzip_eager"] = s.gzip_eager;
             d["gzip_lazy"] = s.gzip_lazy;
             d["gzip_unused"] = s.gzip_unused;
             d["gzip_predicted"] = s.gzip_predicted;
             d["kfd_files_open"] = s.kfd_files_open;
             d["kfd_reads_cached"] = s.kfd_reads_cached;
             d["device_errors"] = s.device_errors;
             d["device_timeouts"] = s.device_timeouts;
             d["sample_count"] = s.sample_hist.count;
             d["sample_sum_s"] = s.sample_hist.sum;
             d["attribution_cache_hits"] = s.attribution_cache_hits;
             d["attribution_cache_misses"] = s.attribution_cache_misses;
             return d;
           })
      .def("scrape_quantile", &Exporter::scrape_quantile)
      .def("scrape_count", &Exporter::scrape_count, "/metrics requests served so far")
      .def("scrape_durations_since", &Exporter::scrape_durations_since, py::arg("from"),
           "server-side service times (s) of the /metrics requests numbered >= from (last 16384)")
      .def("sample_quantile", &Exporter::sample_quantile)
      .def("set_container_meta",
           [](Exporter& e, const py::list& metas) {
             std::vector<ContainerMeta> v;
             for (auto it : metas) {
               py::dict d = it.cast<py::dict>();
               ContainerMeta c;
               get(d, "container_id", &c.container_id);
               get(d, "container_name", &c.container_name);
               get(d, "pod_name", &c.pod_name);
               get(d, "pod_namespace", &c.pod_namespace);
               get(d, "pod_uid", &c.pod_uid);
               get(d, "user_name", &c.user_name);
               c.labels = str_map(d, "labels");
               v.push_back(std::move(c));
             }
             e.set_container_meta(std::move(v));
           })
      .def("set_allocations",
           [](Exporter& e, const py::list& allocs) {
             std::vector<Allocation> v;
             for (auto it : allocs) {
               py::dict d = it.cast<py::dict>();
               Allocation a;
               get(d, "pod_namespace", &a.pod_namespace);
               get(d, "pod_name", &a.pod_name);
               get(d, "container_name", &a.container_name);
               get(d, "container_id", &a.container_id);
               get(d, "pod_uid", &a.pod_uid);
               get(d, "gpu_index", &a.gpu_index);
               get(d, "user_name", &a.user_name);
               a.labels = str_map(d, "labels");
               v.push_back(std::move(a));
             }
             e.set_allocations(std::move(v));
           })
      .def("set_extra",
           [](Exporter& e, const std::string& source, const py::list& series) {
             std::vector<ExtraSeries> v;
             for (auto it : series) {
               py::dict d = it.cast<py::dict>();
               ExtraSeries s;
               get(d, "name", &s.name);
               get(d, "help", &s.help);
               get(d, "type", &s.type);
               get(d, "dev", &s.dev);
               get(d, "value", &s.value);
               for (auto kv : str_map(d, "labels")) s.labels.emplace_back(kv.first, kv.second);
               v.push_back(std::move(s));
             }
             e.set_extra(source, std::move(v));
           })
      .def("resolve_pid",
           [](Exporter& e, uint32_t pid) {
             ProcIdentity id = e.attributor().resolve(pid);
             py::dict d;
             d["valid"] = id.valid;
             d["pid_mismatch"] = id.pid_mismatch;
             d["in_container"] = id.in_container;
             d["opted_in"] = id.opted_in;
             d["comm"] = id.comm;
             d["starttime"] = id.starttime;
             d["runtime"] = id.runtime;
             d["container_id"] = id.container_id;
             d["container_name"] = id.container_name;
             d["pod_name"] = id.pod_name;
             d["pod_namespace"] = id.pod_namespace;
             d["pod_uid"] = id.pod_uid;
             d["user_name"] = id.user_name;
             d["source"] = id.source;
             return d;
           })
      .def("derive_user",
           [](Exporter& e, const std::string& pod, const py::dict& labels) {
             std::map<std::string, std::string> m;
             for (auto kv : labels) m[kv.first.cast<std::string>()] = kv.second.cast<std::string>();
             return e.attributor().derive_user(pod, m);
           })
      .def("mock_set_util", [](Exporter& e, int dev, double pct) { mock_of(e)->set_util(dev, pct); })
      .def("mock_add_ecc",
           [](Exporter& e, int dev, const std::string& block, uint64_t ue, uint64_t ce, uint64_t de) {
             mock_of(e)->add_ecc(dev, block, ue, ce, de);
           },
           py::arg("dev"), py::arg("block"), py::arg("ue") = 0, py::arg("ce") = 0, py::arg("de") = 0)
      .def("mock_set_ras_event",
           [](Exporter& e, int dev, const std::string& ev, double v) { mock_of(e)->set_ras_event(dev, ev, v); })
      .def("mock_set_procs",
           [](Exporter& e, const py::list& procs) {
             std::vector<MockProc> v;
             for (auto p : procs) v.push_back(mock_proc_from(p.cast<py::dict>()));
             mock_of(e)->set_procs(v);
           })
      .def("mock_set_fail", [](Exporter& e, int dev, int every) { mock_of(e)->set_fail(dev, every); })
      .def("mock_set_hang_ms", [](Exporter& e, double ms, int dev) { mock_of(e)->set_hang_ms(ms, dev); },
           py::arg("ms"), py::arg("dev") = -1)
      .def("mock_set_xgmi",
           [](Exporter& e, int dev, int link, double gbps) { mock_of(e)->set_xgmi(dev, link, gbps); })
      .def("mock_calls", [](Exporter& e, int dev) { return mock_of(e)->calls(dev); })
      .def("mock_prewarms", [](Exporter& e, int dev) { return mock_of(e)->prewarms(dev); })
      .def("mock_set_link_up",
           [](Exporter& e, int dev, int link, bool up) { mock_of(e)->set_link_up(dev, link, up); })
      .def("mock_link_calls", [](Exporter& e, int dev) { return mock_of(e)->link_calls(dev); })
      .def("mock_set_link_fail",
           [](Exporter& e, int dev, bool fail) { mock_of(e)->set_link_fail(dev, fail); })
      .def("mock_fail_scans", [](Exporter& e, int dev, int n) { mock_of(e)->fail_scans(dev, n); })
      .def("mock_fail_procs", [](Exporter& e, int dev, int n) { mock_of(e)->fail_procs(dev, n); })
      .def(
          "time_process_lists",
          [](Exporter& e, int dev, int n) {
            // n back-to-back Backend::processes() calls of one device (a sampler must not be
            // running): the tick's process-list phase in isolation, in microseconds per call
            Backend* b = e.backend();
            if (!b || dev < 0 || dev >= b->device_count()) throw std::runtime_error("no such device");
            if (e.config().interval_s > 0 || e.config().sample_threads != 0)
              throw std::runtime_error("time_process_lists needs interval_s 0 and sample_threads 0 (no concurrent lists)");
            std::vector<double> us;
            size_t rows = 0;
            {
              py::gil_scoped_release nogil;
              std::vector<ProcSample> p;
              for (int k = 0; k < n; ++k) {
                const int64_t t = mono_ns();
                b->processes(dev, &p);
                us.push_back((mono_ns() - t) * 1e-3);
                rows = p.size();
              }
            }
            py::dict d;
            d["us"] = us;
            d["rows"] = rows;
            return d;
          },
          py::arg("dev") = 0, py::arg("n") = 200)
      .def("mock_set_firmware_frozen",
           [](Exporter& e, int dev, bool frozen) { mock_of(e)->set_firmware_frozen(dev, frozen); })
      .def("mock_set_occ_series",
           [](Exporter& e, int dev, const std::vector<double>& v) { mock_of(e)->set_occ_series(dev, v); })
      .def("mock_occ_reads", [](Exporter& e, int dev) { return mock_of(e)->occ_reads(dev); })
      .def("set_device_mfma_util", &Exporter::set_device_mfma_util,
           "per-device wall-time MFMA utilisation (what the PMC sampler publishes)");

  // Native on-device samplers (csrc/core/ondevice.h): the same PMC / probe plugins the standalone
  // binary dlopen()s, driven from C++ threads instead of the Python runners in gpumon/ops.
  py::class_<OnDevice>(m, "OnDevice")
      .def(py::init([](Exporter& e, const NativeOptions& o) { return new OnDevice(&e, o.od); }), py::keep_alive<1, 2>(),
           "the on-device samplers of finalized Options (enable_pmc / enable_probe and their cadence)")
      .def(py::init([](Exporter& e, const py::dict& cfg) { return new OnDevice(&e, ondevice_from(cfg)); }),
           py::keep_alive<1, 2>())
      .def("start",
           [](OnDevice& o) {
             std::string err;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = o.start(&err);
             }
             if (!ok) throw std::runtime_error("on-device samplers: " + err);
           })
      .def("stop",
           [](OnDevice& o) {
             py::gil_scoped_release nogil;
             o.stop();
           })
      .def("step",
           [](OnDevice& o) {
             py::gil_scoped_release nogil;
             return o.step();
           })
      .def("stats", [](const OnDevice& o) {
        auto s = o.stats();
        py::dict d;
        d["pmc_samples"] = s.pmc_samples;
        d["pmc_steps"] = s.pmc_steps;
        d["probe_steps"] = s.probe_steps;
        d["pmc_errors"] = s.pmc_errors;
        d["pmc_resets"] = s.pmc_resets;
        d["pmc_continuous"] = s.pmc_continuous;
        d["helper_restarts"] = s.helper_restarts;
        d["probe_done"] = s.probe_done;
        d["probe_timeouts"] = s.probe_timeouts;
        d["pmc_agents"] = s.pmc_agents;
        d["probe_devices"] = s.probe_devices;
        d["probe_by_bdf"] = s.probe_by_bdf;
        return d;
      });
  m.def("default_plugin_dir", &default_plugin_dir);
  m.def("ondevice_helper_pid", &ondevice_helper_pid, "pid of the running on-device helper (0: none)");
  m.def(
      "parse_yaml_subset",
      [](const std::string& text) {
        YamlDoc doc;
        std::string err;
        if (!parse_yaml_subset(text, &doc, &err)) throw py::value_error(err);
        py::dict d;
        for (const auto& k : doc.order) d[py::str(k)] = doc.values[k];
        return d;
      },
      "The native exporter's config-file parser (csrc/core/options.cpp): key -> list of strings");
  m.def(
      "pmc_derive",
      [](const py::dict& raw, const py::dict& agent, double window_s) {
        std::map<std::string, PmcReduced> r;
        for (auto kv : raw) {
          py::dict v = kv.second.cast<py::dict>();
          PmcReduced x;
          get(v, "sum", &x.sum);
          get(v, "max", &x.max);
          get(v, "n", &x.n);
          get(v, "by_xcc", &x.by_xcc);
          r[kv.first.cast<std::string>()] = x;
        }
        PmcAgentInfo a;
        get(agent, "cu_count", &a.cu_count);
        get(agent, "simd_count", &a.simd_count);
        get(agent, "num_xcc", &a.num_xcc);
        get(agent, "max_waves_per_cu", &a.max_waves_per_cu);
        PmcDerived d = pmc_derive(r, a, window_s);
        py::dict out;
        auto put = [&](const char* k, double v) {
          if (v == v) out[k] = v;
        };
        put("mfma_busy", d.mfma_busy);
        put("occupancy", d.occupancy);
        put("gui_active", d.gui_active);
        if (!d.xcd_mfma_busy.empty()) out["xcd_mfma_busy"] = d.xcd_mfma_busy;
        if (!d.mfma_tflops.empty()) {
          py::dict tf;
          for (const auto& [dt, v] : d.mfma_tflops) tf[py::str(dt)] = v;
          out["mfma_tflops"] = tf;
        }
        return out;
      },
      py::arg("raw"), py::arg("agent"), py::arg("window_s") = 0.0,
      "C++ twin of tests/oracles/ops/pmc.py derive (used by the native samplers)");
}
