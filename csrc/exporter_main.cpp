// gpumon-exporter: standalone native exporter binary (no Python needed).
//
// Reference entrypoint: `python3 /gpu.py` (/root/reference/Dockerfile:7) reading NODE_NAME and
// INFLUXDB_URL from the environment (gpu.py:19-26) and looping forever (gpu.py:258-263).
// Configuration (csrc/core/options.h, the one implementation `gpumon serve` shares): defaults <
// YAML file (--config / GPUMON_CONFIG, the DaemonSet's ConfigMap format) < environment (NODE_NAME,
// INFLUXDB_URL, GPUMON_<KEY>) < --compat < flags. Attribution uses /proc plus the native kubelet
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
  // generated from the one flag table (csrc/core/options.cpp option_flags)
  std::string u = "usage: gpumon-exporter [--config FILE] [--compat] [--print-config] [--once] [flags]\n";
  for (const auto& f : option_flags()) {
    std::string names = f.flag;
    for (const auto& a : split(f.aliases, ','))
      if (!a.empty()) names += ", " + a;
    if (!f.fixed) names += " VALUE";
    char line[512];
    snprintf(line, sizeof line, "  %-44s %s\n", names.c_str(), f.help);
    u += line;
  }
  u += "config keys: docs/configuration.md, in the file (--config / GPUMON_CONFIG, under `gpumon:`), as\n"
       "GPUMON_<KEY> in the environment, or as the flags above; NODE_NAME and INFLUXDB_URL as in the reference\n";
  fputs(u.c_str(), stderr);
}

int main(int argc, char** argv) {
  NativeOptions o;
  std::string err;
  std::vector<std::string> args(argv + 1, argv + argc), rest, warnings;
  // defaults < file < environment < --compat < flags: options_parse (the one implementation)
  switch (options_parse(&o, args, environ, &rest, &warnings, &err)) {
    case ParseStatus::kOk:
      break;
    case ParseStatus::kBadFile:
      fprintf(stderr, "config: %s\n", err.c_str());
      return 2;
    case ParseStatus::kBadEnv:
      fprintf(stderr, "environment: %s\n", err.c_str());
      return 2;
    case ParseStatus::kBadFlag:
      fprintf(stderr, "%s\n", err.c_str());
      usage();
      return 2;
    case ParseStatus::kBadValue:
      fprintf(stderr, "%s\n", err.c_str());
      return 2;
  }
  for (const auto& w : warnings) fprintf(stderr, "%s\n", w.c_str());
  bool once = false, print_config = false;
  for (const auto& a : rest) {
    if (a == "--once") once = true;
    else if (a == "--print-config") print_config = true;
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
  g_log_level = options_log_level(o);
  if (const std::string verr = options_validate(o); !verr.empty()) {
    fprintf(stderr, "config: %s\n", verr.c_str());
    return 2;
  }
  ExporterConfig& cfg = o.cfg;
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
