// gpumon-exporter: standalone native exporter binary (no Python needed).
//
// Reference entrypoint: `python3 /gpu.py` (/root/reference/Dockerfile:7) reading NODE_NAME and
// INFLUXDB_URL from the environment (gpu.py:19-26) and looping forever (gpu.py:258-263).
// Same env names are honoured here; flags override. Attribution in this binary uses /proc
// (cgroup -> container id; HOSTNAME / service-account namespace fallback). The Python CLI
// (`gpumon serve`) adds CRI + kubelet PodResources metadata on top of the same core.
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>

#include "core/common.h"
#include "core/exporter.h"
#include "core/ondevice.h"

using namespace gpumon;

static std::atomic<bool> g_stop{false};
static void on_signal(int) { g_stop = true; }

static void usage() {
  fprintf(stderr,
          "usage: gpumon-exporter [--backend auto|amdsmi|rocm_smi|mock[:k=v,..]] [--interval SEC]\n"
          "                       [--listen ADDR:PORT] [--host NAME] [--devices 0,1,..] [--no-fast-path]\n"
          "                       [--sysfs /sys] [--influx-url URL] [--influx-extended] [--influx-schema 2018|2019]\n"
          "                       [--opt-in-label KEY=VALUE] [--user-regex RE] [--user-label KEY]\n"
          "                       [--pod-labels KEY,KEY..]\n"
          "                       [--procfs /proc] [--no-processes] [--ras-every TICKS] [--no-gzip] [--sample-threads N]\n"
          "                       [--http-threads N] [--log-level debug|info|warn|error] [--roctx] [--once]\n"
          "                       [--pod-resources SOCKET | --no-pod-resources] [--cri SOCKET | --no-cri]\n"
          "                       [--dra-drivers gpu.amd.com,..|none]\n"
          "                       [--pmc] [--pmc-counters A,B,..] [--pmc-window SEC] [--probe] [--probe-every N]\n"
          "                       [--probe-blocks N] [--plugin-dir DIR]\n"
          "env: NODE_NAME, INFLUXDB_URL, GPUMON_LISTEN, GPUMON_INTERVAL, GPUMON_BACKEND\n");
}

int main(int argc, char** argv) {
  ExporterConfig cfg;
  if (const char* v = getenv("NODE_NAME")) cfg.host = v;
  if (const char* v = getenv("INFLUXDB_URL")) cfg.influx_url = v;
  if (const char* v = getenv("GPUMON_BACKEND")) cfg.backend = v;
  if (const char* v = getenv("GPUMON_INTERVAL")) cfg.interval_s = atof(v);
  std::string listen = getenv("GPUMON_LISTEN") ? getenv("GPUMON_LISTEN") : "0.0.0.0:9400";
  bool once = false;
  OnDeviceConfig od;
  int probe_every = 1;
  // kubelet PodResources: on by default when the socket is mounted (deploy/k8s DaemonSet)
  std::string podres = "/var/lib/kubelet/pod-resources/kubelet.sock";
  std::string cri;  // "" = first existing well-known runtime socket, "none" = off
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        usage();
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--backend") cfg.backend = next();
    else if (a == "--interval") cfg.interval_s = atof(next().c_str());
    else if (a == "--listen") listen = next();
    else if (a == "--host") cfg.host = next();
    else if (a == "--devices") {
      for (const auto& s : split(next(), ','))
        if (!s.empty()) cfg.devices.push_back(atoi(s.c_str()));
    } else if (a == "--influx-url") cfg.influx_url = next();
    else if (a == "--influx-extended") cfg.influx_extended = true;
    else if (a == "--influx-schema") cfg.influx_schema = atoi(next().c_str());
    else if (a == "--no-fast-path") cfg.fast_path = false;
    else if (a == "--sysfs") cfg.sysfs_root = next();
    else if (a == "--roctx") cfg.roctx = true;
    else if (a == "--pod-resources") podres = next();
    else if (a == "--no-pod-resources") podres = "";
    else if (a == "--cri") cri = next();
    else if (a == "--no-cri") cri = "none";
    else if (a == "--dra-drivers") {
      const std::string v = next();
      cfg.pod_resources_dra_drivers.clear();
      if (v != "none")
        for (const auto& d : split(v, ','))
          if (!d.empty()) cfg.pod_resources_dra_drivers.push_back(d);
    }
    else if (a == "--opt-in-label") cfg.attribution.opt_in = next();
    else if (a == "--user-regex") cfg.attribution.user_regex = next();
    else if (a == "--pod-labels") cfg.attribution.label_allowlist = split(next(), ',');
    else if (a == "--user-label") cfg.attribution.user_label = next();
    else if (a == "--procfs") cfg.attribution.procfs_root = next();
    else if (a == "--no-processes") cfg.processes = false;
    else if (a == "--ras-every") cfg.ras_every = atoi(next().c_str());
    else if (a == "--no-gzip") cfg.gzip = false;
    else if (a == "--sample-threads") cfg.sample_threads = atoi(next().c_str());
    else if (a == "--http-threads") cfg.http_threads = atoi(next().c_str());
    else if (a == "--once") once = true;
    else if (a == "--pmc") od.pmc = true;
    else if (a == "--pmc-counters") od.pmc_counters = split(next(), ',');
    else if (a == "--pmc-window") od.pmc_window_s = atof(next().c_str());
    else if (a == "--probe") od.probe = true;
    else if (a == "--probe-every") probe_every = std::max(1, atoi(next().c_str()));
    else if (a == "--probe-blocks") od.probe_blocks = atoi(next().c_str());
    else if (a == "--plugin-dir") od.plugin_dir = next();
    else if (a == "--log-level") {
      std::string l = next();
      g_log_level = l == "debug" ? 0 : l == "info" ? 1 : l == "warn" ? 2 : 3;
    } else if (a == "-h" || a == "--help") {
      usage();
      return 0;
    } else {
      fprintf(stderr, "unknown flag %s\n", a.c_str());
      usage();
      return 2;
    }
  }
  size_t colon = listen.rfind(':');
  cfg.listen_addr = colon == std::string::npos ? "0.0.0.0" : listen.substr(0, colon);
  cfg.port = atoi(colon == std::string::npos ? listen.c_str() : listen.c_str() + colon + 1);
  if (cfg.host.empty()) cfg.host = "no_name";
  if (!podres.empty() && access(podres.c_str(), F_OK) == 0) cfg.pod_resources_socket = podres;
  if (cri.empty()) {
    for (const char* c : {"/run/containerd/containerd.sock", "/var/run/crio/crio.sock", "/run/crio/crio.sock",
                          "/var/run/cri-dockerd.sock"})
      if (access(c, F_OK) == 0) {
        cri = c;
        break;
      }
  }
  if (!cri.empty() && cri != "none") cfg.cri_socket = cri;
  // on-device samplers run at the sampler cadence (the probe every N ticks)
  const double period = cfg.interval_s > 0 ? std::max(cfg.interval_s, 0.1) : 1.0;
  od.pmc_every_s = period;
  od.probe_every_s = period * probe_every;

  if (once) {
    cfg.serve_http = false;
    cfg.interval_s = 0;
    Exporter e(cfg);
    std::string err;
    if (!e.start(&err)) {
      fprintf(stderr, "start failed: %s\n", err.c_str());
      return 1;
    }
    OnDevice ondev(&e, od);
    if ((od.pmc || od.probe) && !ondev.start(&err)) {
      fprintf(stderr, "on-device samplers: %s\n", err.c_str());
      return 1;
    }
    ondev.step();
    e.tick();  // second tick so rates are populated (and the on-device series are rendered)
    auto s = e.snapshot();
    fwrite(s->body.data(), 1, s->body.size(), stdout);
    e.stop();
    return 0;
  }

  signal(SIGINT, on_signal);
  signal(SIGTERM, on_signal);
  signal(SIGPIPE, SIG_IGN);
  Exporter e(cfg);
  std::string err;
  if (!e.start(&err)) {
    fprintf(stderr, "start failed: %s\n", err.c_str());
    return 1;
  }
  if (!err.empty()) GPUMON_LOG(LogLevel::kWarn, "main", "backend not ready (retrying): " + err);
  OnDevice ondev(&e, od);
  if (od.pmc || od.probe) {
    std::string oerr;
    if (!ondev.start(&oerr)) {
      // fail loudly: a DaemonSet asked for PMC / probe series and would otherwise silently lack them
      fprintf(stderr, "on-device samplers: %s\n", oerr.c_str());
      e.stop();
      return 1;
    }
  }
  GPUMON_LOG(LogLevel::kInfo, "main",
             "serving http://" + cfg.listen_addr + ":" + std::to_string(e.port()) +
                 "/metrics host=" + cfg.host + " interval=" + std::to_string(cfg.interval_s) + "s");
  while (!g_stop) std::this_thread::sleep_for(std::chrono::milliseconds(200));
  ondev.stop();
  e.stop();
  return 0;
}
