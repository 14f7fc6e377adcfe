// gpumon-exporter: standalone native exporter binary (no Python needed).
//
// Reference entrypoint: `python3 /gpu.py` (/root/reference/Dockerfile:7) reading NODE_NAME and
// INFLUXDB_URL from the environment (gpu.py:19-26) and looping forever (gpu.py:258-263).
// Configuration (csrc/core/options.h) uses the Python control plane's keys and precedence:
// defaults < YAML file (--config / GPUMON_CONFIG, the DaemonSet's ConfigMap format) < environment
// (NODE_NAME, INFLUXDB_URL, GPUMON_<KEY>) < flags. Attribution uses /proc plus the native kubelet
// PodResources and CRI pollers; --pmc / --probe load the on-device plugins.
#include <signal.h>
#include <sys/resource.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#include "core/common.h"
#include "core/exporter.h"
#include "core/ondevice.h"
#include "core/options.h"
#include "core/tls.h"

using namespace gpumon;

extern char** environ;

static std::atomic<bool> g_stop{false}, g_hup{false};
static void on_signal(int) { g_stop = true; }
static void on_hup(int) { g_hup = true; }

static void usage() {
  fprintf(stderr,
          "usage: gpumon-exporter [--config FILE] [--print-config] [--once]\n"
          "                       [--backend auto|amdsmi|rocm_smi|mock[:k=v,..]] [--interval SEC]\n"
          "                       [--listen HOST:PORT|[V6]:PORT|:PORT] [--host NAME] [--devices 0,1|BDF,..] [--no-fast-path]\n"
          "                       [--sysfs /sys] [--influx-url URL] [--influx-extended] [--influx-schema 2018|2019]\n"
          "                       [--influx-ca-file PEM] [--influx-tls-insecure] [--influx-client-cert PEM --influx-client-key PEM]\n"
          "                       [--tls-cert-file PEM --tls-key-file PEM [--tls-client-ca-file PEM]]  (/metrics over HTTPS)\n"
          "                       [--http-auth-token-file FILE]  (/metrics needs Authorization: Bearer <token>)\n"
          "                       [--opt-in-label KEY=VALUE] [--user-regex RE] [--user-label KEY]\n"
          "                       [--pod-labels KEY,KEY..]\n"
          "                       [--procfs /proc] [--no-processes] [--ras-every TICKS] [--ras-slices N] [--no-gzip] [--metrics-include GLOBS] [--metrics-exclude GLOBS] [--sample-threads N] [--rt-priority N] [--prewarm-ms MS]\n"
          "                       [--http-threads N] [--log-level debug|info|warn|error] [--roctx]\n"
          "                       [--pod-resources SOCKET | --no-pod-resources] [--cri SOCKET | --no-cri] [--docker SOCKET]\n"
          "                       [--pod-logs /var/log] [--device-checkpoint FILE]\n"
          "                       [--dra-drivers gpu.amd.com,..|none]\n"
          "                       [--pmc] [--pmc-counters A,B,..] [--pmc-mode continuous|window] [--pmc-window SEC] [--probe] [--probe-every N]\n"
          "                       [--probe-blocks N] [--plugin-dir DIR] [--device-timeout SEC]\n"
          "                       [--control-plane native|off] [--compat]\n"
          "the Python entry point's spellings work too: --procfs-root, --sysfs-root, --cri-socket,\n"
          "--pod-resources-socket, --docker-socket, --pod-log-root, --enable-pmc, --enable-probe-kernel\n"
          "config keys: the gpumon.* keys of gpumon/config.py (docs/configuration.md), in the file, as\n"
          "GPUMON_<KEY> in the environment, or as the flags above; NODE_NAME and INFLUXDB_URL as in the reference\n");
}

int main(int argc, char** argv) {
  NativeOptions o;
  std::string err;
  // 1. config file: --config wins over GPUMON_CONFIG
  const char* config_env = getenv("GPUMON_CONFIG");
  std::string config = config_env ? config_env : "";
  for (int i = 1; i + 1 < argc; ++i)
    if (std::string(argv[i]) == "--config") config = argv[i + 1];
  if (!config.empty()) {
    std::vector<std::string> unknown;
    if (!options_load_file(&o, config, &unknown, &err)) {
      fprintf(stderr, "config: %s\n", err.c_str());
      return 2;
    }
    for (const auto& k : unknown)
      fprintf(stderr, "config: key '%s' is not used by the native exporter (ignored)\n", k.c_str());
  }
  // 2. environment
  if (!options_apply_env(&o, environ, &err)) {
    fprintf(stderr, "environment: %s\n", err.c_str());
    return 2;
  }
  // 3. flags
  bool once = false, print_config = false, compat = false;
  auto set = [&](const char* key, const std::string& v) {
    std::string e;
    if (options_set(&o, key, {v}, &e) < 0) {
      fprintf(stderr, "%s\n", e.c_str());
      exit(2);
    }
  };
  // --compat (the reference's behaviour: opt-in label mlgpu=mlgpu, 10 s interval) sits between the
  // environment and the flags, as in gpumon/config.py from_args: explicit flags still win
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--compat") compat = true;
  if (compat) {
    if (o.cfg.attribution.opt_in.empty()) set("opt_in_label", "mlgpu=mlgpu");
    set("interval", "10");
  }
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        usage();
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--config") next();
    else if (a == "--print-config") print_config = true;
    else if (a == "--once") once = true;
    else if (a == "--backend") set("backend", next());
    else if (a == "--interval") set("interval", next());
    else if (a == "--listen") set("listen", next());
    else if (a == "--host") set("host", next());
    else if (a == "--devices") set("devices", next());
    else if (a == "--influx-url") set("influx_url", next());
    else if (a == "--influx-token") set("influx_token", next());
    else if (a == "--influx-extended") set("influx_extended", "true");
    else if (a == "--influx-gzip") set("influx_gzip", "true");
    else if (a == "--influx-schema") set("influx_schema", next());
    else if (a == "--influx-ca-file") set("influx_ca_file", next());
    else if (a == "--tls-cert-file") set("tls_cert_file", next());
    else if (a == "--tls-key-file") set("tls_key_file", next());
    else if (a == "--tls-client-ca-file") set("tls_client_ca_file", next());
    else if (a == "--http-auth-token-file") set("http_auth_token_file", next());
    else if (a == "--influx-tls-insecure") set("influx_tls_insecure", "true");
    else if (a == "--influx-client-cert") set("influx_client_cert", next());
    else if (a == "--influx-client-key") set("influx_client_key", next());
    else if (a == "--no-fast-path") set("fast_path", "false");
    else if (a == "--sysfs" || a == "--sysfs-root") set("sysfs_root", next());
    else if (a == "--roctx") set("roctx", "true");
    else if (a == "--pod-resources" || a == "--pod-resources-socket") set("pod_resources_socket", next());
    else if (a == "--no-pod-resources") set("pod_resources_socket", "");
    else if (a == "--cri" || a == "--cri-socket") set("cri_socket", next());
    else if (a == "--no-cri") set("cri_socket", "none");
    else if (a == "--docker" || a == "--docker-socket") set("docker_socket", next());
    else if (a == "--pod-logs" || a == "--pod-log-root") set("pod_log_root", next());
    else if (a == "--device-checkpoint") set("device_checkpoint", next());
    else if (a == "--dra-drivers") {
      const std::string v = next();
      set("dra_drivers", v == "none" ? "" : v);
    } else if (a == "--control-plane") {
      // off: no kubelet / CRI / Docker / log-tree metadata pollers (the Python entry point's flag)
      const std::string v = next();
      if (v == "off") {
        for (const char* k : {"pod_resources_socket", "docker_socket", "pod_log_root", "device_checkpoint"}) set(k, "");
        set("cri_socket", "none");
      } else if (v != "native") {
        fprintf(stderr, "--control-plane: native or off, not '%s'\n", v.c_str());
        return 2;
      }
    } else if (a == "--compat") {
      // applied before the flags (above)
    } else if (a == "--opt-in-label") set("opt_in_label", next());
    else if (a == "--user-regex") set("user_regex", next());
    else if (a == "--user-label") set("user_label", next());
    else if (a == "--pod-labels") set("pod_label_allowlist", next());
    else if (a == "--procfs" || a == "--procfs-root") set("procfs_root", next());
    else if (a == "--no-processes") set("processes", "false");
    else if (a == "--ras-every") set("ras_every", next());
    else if (a == "--ras-slices") set("ras_slices", next());
    else if (a == "--no-gzip") set("gzip", "false");
    else if (a == "--device-timeout") set("device_timeout_s", next());
    else if (a == "--metrics-include") set("metrics_include", next());
    else if (a == "--metrics-exclude") set("metrics_exclude", next());
    else if (a == "--sample-threads") set("sample_threads", next());
    else if (a == "--rt-priority") set("rt_priority", next());
    else if (a == "--http-rt-priority") set("http_rt_priority", next());
    else if (a == "--prewarm-ms") set("prewarm_ms", next());
    else if (a == "--http-threads") set("http_threads", next());
    else if (a == "--log-level") set("log_level", next());
    else if (a == "--pmc" || a == "--enable-pmc") set("enable_pmc", "true");
    else if (a == "--pmc-counters") set("pmc_counters", next());
    else if (a == "--pmc-window") o.od.pmc_window_s = atof(next().c_str());
    else if (a == "--pmc-mode") set("pmc_mode", next());
    else if (a == "--probe" || a == "--enable-probe-kernel") set("enable_probe", "true");
    else if (a == "--probe-every") set("probe_every", next());
    else if (a == "--probe-blocks") o.od.probe_blocks = atoi(next().c_str());
    else if (a == "--plugin-dir") set("plugin_dir", next());
    else if (a == "-h" || a == "--help") {
      usage();
      return 0;
    } else {
      fprintf(stderr, "unknown flag %s\n", a.c_str());
      usage();
      return 2;
    }
  }
  if (print_config) {
    printf("%s\n", options_json(o).c_str());
    return 0;
  }
  if (!options_finalize(&o, &err)) {
    fprintf(stderr, "config: %s\n", err.c_str());
    return 2;
  }
  ExporterConfig& cfg = o.cfg;
  {
    // an Influx push that cannot work is a startup error, not a silently idle pusher
    TlsOptions t;
    t.ca_file = cfg.influx_ca_file;
    t.insecure = cfg.influx_tls_insecure;
    t.client_cert = cfg.influx_client_cert;
    t.client_key = cfg.influx_client_key;
    const std::string perr = check_push_config(cfg.influx_url, cfg.influx_token, t);
    if (!perr.empty()) {
      fprintf(stderr, "config: %s\n", perr.c_str());
      return 2;
    }
    // /metrics over HTTPS: the certificate, key and client CA must load
    const std::string serr = check_serve_tls(cfg.tls_cert_file, cfg.tls_key_file, cfg.tls_client_ca_file);
    if (!serr.empty()) {
      fprintf(stderr, "config: %s\n", serr.c_str());
      return 2;
    }
    // /metrics behind a bearer token: the token file must hold one
    if (const std::string aerr = check_auth_token_file(cfg.http_auth_token_file); !aerr.empty()) {
      fprintf(stderr, "config: http_auth_token_file: %s\n", aerr.c_str());
      return 2;
    }
  }
  const OnDeviceConfig& od = o.od;

  // The on-device samplers start BEFORE the backend: the PMC helper process is spawned while
  // nothing in this process has touched the GPU yet, and the samplers pick the devices up once the
  // backend lists them (OnDevice maps agents / creates probes on its first steps).
  if (once) {
    // One sample to stdout, over a short live interval (<= 0.5 s): the device workers sub-sample
    // KFD occupancy through it (an interval mean, not one instantaneous read that can land between
    // a tenant's kernels), rates span it, and the on-device step lands before its closing tick.
    cfg.serve_http = false;
    cfg.interval_s = std::min(cfg.interval_s > 0 ? cfg.interval_s : 0.5, 0.5);
    // the on-device values printed are the synchronous step's (PMC over --pmc-window): the
    // samplers' own loops must not read again inside the short interval
    o.od.pmc_every_s = o.od.probe_every_s = 3600.0;
    Exporter e(cfg);
    OnDevice ondev(&e, od);
    if ((od.pmc || od.probe) && !ondev.start(&err)) {
      fprintf(stderr, "on-device samplers: %s\n", err.c_str());
      return 1;
    }
    if (!e.start(&err)) {
      fprintf(stderr, "start failed: %s\n", err.c_str());
      ondev.stop();
      return 1;
    }
    if (!err.empty()) fprintf(stderr, "backend not ready: %s\n", err.c_str());
    ondev.step();
    // the tick after the step renders its series; the one after that spans a whole interval
    // that started after the step
    e.wait_for_seq(e.seq() + 2, 30.0 + 4 * cfg.interval_s);
    auto s = e.snapshot();
    fwrite(s->body.data(), 1, s->body.size(), stdout);
    ondev.stop();
    e.stop();
    return 0;
  }

  signal(SIGINT, on_signal);
  signal(SIGTERM, on_signal);
  signal(SIGPIPE, SIG_IGN);
  signal(SIGHUP, on_hup);  // re-check the TLS files now (a rotated certificate is also found within 5 s)
  // The soft fd limit up to the hard one, as daemons (and Go's runtime) do: container runtimes often
  // leave the soft limit at 1024, and the HTTP connection cap is derived from it. Nothing in the
  // process (or the libraries it loads: libamd_smi, libdrm, OpenSSL) uses select(), so fd numbers
  // past 1024 are safe.
  if (rlimit rl{}; getrlimit(RLIMIT_NOFILE, &rl) == 0 && rl.rlim_cur < rl.rlim_max) {
    const rlim_t was = rl.rlim_cur;
    rl.rlim_cur = rl.rlim_max;
    if (setrlimit(RLIMIT_NOFILE, &rl) == 0)
      GPUMON_LOG(LogLevel::kDebug, "main",
                 "RLIMIT_NOFILE soft limit " + std::to_string(was) + " -> " +
                     (rl.rlim_max == RLIM_INFINITY ? std::string("unlimited") : std::to_string(rl.rlim_max)));
  }
  Exporter e(cfg);
  OnDevice ondev(&e, od);
  if (od.pmc || od.probe) {
    std::string oerr;
    if (!ondev.start(&oerr)) {
      // fail loudly: a DaemonSet asked for PMC / probe series and would otherwise silently lack them
      fprintf(stderr, "on-device samplers: %s\n", oerr.c_str());
      return 1;
    }
  }
  if (!e.start(&err)) {
    fprintf(stderr, "start failed: %s\n", err.c_str());
    ondev.stop();
    return 1;
  }
  if (!err.empty()) GPUMON_LOG(LogLevel::kWarn, "main", "backend not ready (retrying): " + err);
  GPUMON_LOG(LogLevel::kInfo, "main",
             std::string("serving ") + (cfg.tls_cert_file.empty() ? "http://" : "https://") + e.listen_desc() +
                 "/metrics host=" + cfg.host + " interval=" + std::to_string(cfg.interval_s) + "s");
  while (!g_stop) {
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
    if (g_hup.exchange(false)) {
      GPUMON_LOG(LogLevel::kInfo, "main", "SIGHUP: re-checking the TLS files");
      e.reload_tls();
    }
  }
  ondev.stop();
  e.stop();
  return 0;
}
