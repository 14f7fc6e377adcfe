// Loopback-only introspection endpoints (ExporterConfig::debug_listen), served by their own
// one-thread HttpServer so that nothing here shares a loop with /metrics:
//
//   GET /debug/state                    pid, seq, statics, self stats
//   GET /debug/wait?seq=N&timeout_s=T   blocks (this loop only) until the tick with seq >= N is
//                                       published; returns {"seq", "ok"}
//   GET /debug/ticks?since=SEQ          tick log entries with seq > SEQ: phases + per-device values
//   GET /debug/scrapes?since=N          the exact server-side service times of /metrics requests
//                                       numbered >= N (the histogram's ring, exporter.h)
//   GET /debug/samples                  the last tick's per-device fields and interval rates
//   GET /debug/rows                     the last tick's pod_gpu rows
//   GET /debug/procs                    every GPU context of the last tick's process lists and
//                                       whether it became a row (the hidden ones by pid)
//
// What these are for: a bench or test that runs bin/gpumon-exporter as its own process (the
// DaemonSet's ENTRYPOINT) reads the same exact numbers the in-process bindings give
// (csrc/bindings/core_module.cpp), without a Python runtime in the exporter. The reference had no
// endpoint at all (push only, /root/reference/gpu.py:145).
#include <unistd.h>

#include <cstdlib>

#include "common.h"
#include "exporter_internal.h"
#include "json_out.h"

namespace gpumon {

namespace {

std::string query_value(const std::string& q, const char* key) {
  for (const auto& kv : split(q, '&')) {
    const size_t eq = kv.find('=');
    if (eq != std::string::npos && kv.compare(0, eq, key) == 0) return kv.substr(eq + 1);
  }
  return "";
}

void statics_json(const std::vector<DeviceStatic>& st, JsonOut* j) {
  j->arr();
  for (const auto& s : st) {
    j->obj()
        .kv("index", s.index)
        .kv("hip_id", s.hip_id)
        .kv("gpu_id", s.gpu_id)
        .kv("uuid", s.uuid)
        .kv("bdf", s.bdf)
        .kv("model", s.model)
        .kv("gfx_target", s.gfx_target)
        .kv("compute_partition", s.compute_partition)
        .kv("kfd_node", s.kfd_node)
        .kv("partition_id", s.partition_id)
        .kv("num_cu", s.num_cu)
        .kv("driver_version", s.driver_version)
        .kv("vram_total_bytes", s.vram_total_bytes)
        .end_obj();
  }
  j->end_arr();
}

void self_json(const SelfStats& s, JsonOut* j) {
  j->obj()
      .kv("backend", s.backend)
      .kv("backend_version", s.backend_version)
      .kv("backend_up", s.backend_up)
      .kv("fast_path_devices", s.fast_path_devices)
      .kv("ticks", s.ticks)
      .kv("samples", s.samples)
      .kv("stale_samples", s.stale_samples)
      .kv("frozen_samples", s.frozen_samples)
      .kv("overruns", s.overruns)
      .kv("occupancy_reads", s.occupancy_reads)
      .kv("process_list_failures", s.process_list_failures)
      .kv("hidden_contexts", s.hidden_contexts)
      .kv("hidden_peer_contexts", s.hidden_peer_contexts)
      .kv("rt_threads", s.rt_threads)
      .kv("http_rt_loops", s.http_rt_loops)
      .kv("http_connections", s.http_connections)
      .kv("scrapes", s.scrapes)
      .kv("pods_attributed", s.pods_attributed)
      .kv("gzip_eager", s.gzip_eager)
      .kv("gzip_lazy", s.gzip_lazy)
      .kv("cpu_seconds", s.cpu_seconds)
      .kv("rss_bytes", s.rss_bytes)
      .kv("threads", s.threads)
      .kv("open_fds", s.open_fds);
  j->key("backend_calls").obj();
  for (const auto& c : s.backend_calls)
    j->key(c.call.c_str()).obj().kv("n", c.n).kv("errors", c.errors).kv("seconds", c.seconds).end_obj();
  j->end_obj();
  j->key("device_errors").arr();
  for (auto e : s.device_errors) j->u64(e);
  j->end_arr();
  j->end_obj();
}

void tick_json(const TickInfo& t, JsonOut* j) {
  j->obj()
      .kv("seq", t.seq)
      .kv("duration_s", t.duration_s)
      .kv("devices", t.devices)
      .kv("devices_ok", t.devices_ok)
      .kv("pod_rows", t.pod_rows)
      .kv("body_bytes", t.body_bytes)
      .kv("t_sample", t.t_sample)
      .kv("t_procs", t.t_procs)
      .kv("t_attrib", t.t_attrib)
      .kv("t_render", t.t_render)
      .kv("t_gzip", t.t_gzip)
      .kv("t_wake", t.t_wake)
      .kv("t_device", t.t_device)
      .kv("t_late", t.t_late)
      .kv("link_refreshes", t.link_refreshes)
      .kv("ras_reads", t.ras_reads)
      .kv("ras_full", t.ras_full);
  j->key("dev").arr();
  for (const auto& d : t.dev)
    j->obj()
        .kv("ok", d.ok)
        .kv("fresh", d.fresh)
        .kv("rates_valid", d.rates_valid)
        .kv("gfx_util", d.gfx_util)
        .kv("xgmi_wr_Bps", d.xgmi_wr_Bps)
        .kv("xgmi_rd_Bps", d.xgmi_rd_Bps)
        .kv("pcie_Bps", d.pcie_Bps)
        .kv("t_device", d.t_device)
        .kv("t_procs", d.t_procs)
        .end_obj();
  j->end_arr().end_obj();
}

}  // namespace

bool parse_debug_listen(const std::string& listen, std::string* host, int* port, std::string* err) {
  if (!parse_listen(listen, host, port, err)) return false;
  // loopback only: the introspection views name processes, pods and timings of the whole node and
  // carry no authentication (bearer token / TLS guard /metrics only)
  if (*host == "localhost") *host = "127.0.0.1";
  if (!(starts_with(*host, "127.") || *host == "::1")) {
    *err = "debug_listen '" + listen + "': loopback addresses only (127.0.0.0/8 or [::1])";
    return false;
  }
  return true;
}

void Exporter::handle_debug(const HttpRequest& req, HttpResponse* resp) {
  resp->content_type = "application/json";
  JsonOut j;
  if (req.path == "/debug/state") {
    j.obj().kv("pid", static_cast<int64_t>(getpid())).kv("seq", seq()).kv("running", running_.load());
    j.kv("port", port()).kv("scrape_count", scrape_count()).kv("interval_s", cfg_.interval_s);
    j.key("statics");
    statics_json(*statics_ptr(), &j);
    j.key("self");
    self_json(self_stats(), &j);
    j.end_obj();
  } else if (req.path == "/debug/wait") {
    const uint64_t want = strtoull(query_value(req.query, "seq").c_str(), nullptr, 10);
    const std::string ts = query_value(req.query, "timeout_s");
    const double timeout = ts.empty() ? 10.0 : std::min(120.0, std::max(0.0, atof(ts.c_str())));
    const bool ok = wait_for_seq(want, timeout);
    j.obj().kv("seq", seq()).kv("ok", ok).end_obj();
  } else if (req.path == "/debug/ticks") {
    const uint64_t since = strtoull(query_value(req.query, "since").c_str(), nullptr, 10);
    j.arr();
    for (const auto& t : tick_log())
      if (t.seq > since) tick_json(t, &j);
    j.end_arr();
  } else if (req.path == "/debug/scrapes") {
    const uint64_t since = strtoull(query_value(req.query, "since").c_str(), nullptr, 10);
    const uint64_t count = scrape_count();
    j.obj().kv("count", count).key("durations_s").arr();
    for (float d : scrape_durations_since(since)) j.num(d);
    j.end_arr().end_obj();
  } else if (req.path == "/debug/samples") {
    auto st = state_ptr();
    j.arr();
    for (size_t i = 0; i < st->samples.size(); ++i) {
      const DeviceSample& s = st->samples[i];
      j.obj().kv("index", static_cast<int64_t>(i)).kv("ok", s.ok).kv("fresh", s.fresh).key("fields").obj();
      for (int f = 0; f < F_COUNT; ++f) j.kv(field_name(f), s.v[f]);
      j.end_obj();
      if (i < st->rates.size()) {
        const DeviceRates& r = st->rates[i];
        j.key("rates").obj().kv("valid", r.valid).kv("dt_s", r.dt_s).kv("pcie_Bps", r.pcie_Bps);
        j.kv("gfx_activity_avg_pct", r.gfx_activity_avg_pct).kv("power_from_energy_w", r.power_from_energy_w);
        j.key("xgmi_wr_Bps").arr();
        for (int k = 0; k < r.n_links; ++k) j.num(r.xgmi_wr_Bps[k]);
        j.end_arr().key("xgmi_rd_Bps").arr();
        for (int k = 0; k < r.n_links; ++k) j.num(r.xgmi_rd_Bps[k]);
        j.end_arr().end_obj();
      }
      j.end_obj();
    }
    j.end_arr();
  } else if (req.path == "/debug/rows") {
    auto st = state_ptr();
    j.arr();
    for (const auto& r : st->rows)
      j.obj()
          .kv("dev", r.dev)
          .kv("idle", r.idle)
          .kv("pid", r.pid)
          .kv("procname", r.procname)
          .kv("namespace", r.pod_namespace)
          .kv("podname", r.pod_name)
          .kv("container", r.container)
          .kv("containerid", r.containerid)
          .kv("user_name", r.user_name)
          .kv("used_memory_bytes", r.used_memory_bytes)
          .kv("gpu_util", r.gpu_util)
          .kv("proc_gfx_util", r.proc_gfx_util)
          .kv("cu_occupancy", r.cu_occupancy)
          .kv("occ_samples", r.occ_samples)
          .kv("queues", r.queues)
          .kv("mfma_util", r.mfma_util)
          .end_obj();
    j.end_arr();
  } else if (req.path == "/debug/procs") {
    // every GPU context of the last tick's process lists, and whether it became a pod_gpu row: the
    // ones that did not are the hidden empty / peer contexts (or not opted in), named by pid
    auto st = state_ptr();
    j.arr();
    for (size_t d = 0; d < st->procs.size(); ++d)
      for (const auto& p : st->procs[d]) {
        bool row = false;
        for (const auto& r : st->rows)
          if (!r.idle && r.dev == static_cast<int>(d) && r.pid == std::to_string(p.pid)) row = true;
        const char* why = row ? "" : "merged";  // a second KFD context of a pid that has its row
        for (const auto& h : st->hidden)
          if (h.dev == static_cast<int>(d) && h.pid == p.pid) why = h.why;
        j.obj()
            .kv("dev", static_cast<int64_t>(d))
            .kv("pid", static_cast<int64_t>(p.pid))
            .kv("vram_bytes", p.vram_bytes)
            .kv("mem_bytes", p.mem_bytes)
            .kv("cu_occupancy", p.cu_occupancy)
            .kv("occ_samples", static_cast<int64_t>(p.occ_samples))
            .kv("occ_busy", static_cast<int64_t>(p.occ_busy))
            .kv("queues", static_cast<int64_t>(p.queues))
            .kv("row", row)
            .kv("why", why)
            .end_obj();
      }
    j.end_arr();
  } else {
    resp->status = 404;
    resp->content_type = "text/plain; charset=utf-8";
    resp->inline_body = "not found\n";
    return;
  }
  resp->inline_body = j.take();
  resp->inline_body.push_back('\n');
}

std::string Exporter::debug_view(const std::string& path_and_query) {
  HttpRequest req;
  req.method = "GET";
  const size_t q = path_and_query.find('?');
  req.path = path_and_query.substr(0, q);
  if (q != std::string::npos) req.query = path_and_query.substr(q + 1);
  HttpResponse resp;
  handle_debug(req, &resp);
  return resp.status == 200 ? resp.inline_body : std::string();
}

}  // namespace gpumon
