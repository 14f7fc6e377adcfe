// lib/gpumon-ondevice-helper: runs the exporter's on-device samplers' GPU-runtime side -- the
// rocprofiler-sdk device counting contexts and the K1 probe (protocol and rationale:
// ondevice_helper_proto.h). Reads requests on fd 0, answers on fd 1. Links libgpumon_pmc.so
// (rpath $ORIGIN); dlopen()s libgpumon_probe.so from its own directory on the first probe request,
// so a PMC-only helper never loads HIP and PMC initialisation (which must precede HSA's) comes
// first whenever both are used. Exits on EOF, on QUIT, and with its parent (PR_SET_PDEATHSIG
// SIGKILL: a frozen helper cannot act on SIGTERM).
#include <dlfcn.h>
#include <sys/prctl.h>
#include <unistd.h>

#include <time.h>

#include <algorithm>
#include <cerrno>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ondevice_abi.h"
#include "ondevice_helper_proto.h"

namespace {

bool read_full(int fd, void* p, size_t n) {
  auto* b = static_cast<char*>(p);
  while (n) {
    const ssize_t r = ::read(fd, b, n);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    b += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

bool write_full(int fd, const void* p, size_t n) {
  auto* b = static_cast<const char*>(p);
  while (n) {
    const ssize_t r = ::write(fd, b, n);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    b += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

bool reply(int rc, int started, const std::string& err, const void* payload, size_t len) {
  gpumon_pmc_resp_t h{GPUMON_PMC_PROTO_MAGIC, rc, started, static_cast<uint32_t>(err.size()),
                      static_cast<uint32_t>(len)};
  return write_full(1, &h, sizeof h) && write_full(1, err.data(), err.size()) && (!len || write_full(1, payload, len));
}

// libgpumon_probe.so, resolved on first use
struct ProbeLib {
  void* h = nullptr;
  int (*count)() = nullptr;
  gpumon_probe* (*create)(int, int, int, int, char*, size_t) = nullptr;
  int (*launch)(gpumon_probe*) = nullptr;
  int (*wait)(gpumon_probe*, int, double, gpumon_probe_result_t*) = nullptr;
  void (*destroy)(gpumon_probe*) = nullptr;
  size_t (*pci)(int, char*, size_t) = nullptr;  // optional
  std::vector<gpumon_probe*> handles;  // handle id = index
};
ProbeLib g_probe;
bool g_pmc_used = false;

bool probe_lib(std::string* err) {
  if (g_probe.h) return true;
  char self[4096];
  const ssize_t n = readlink("/proc/self/exe", self, sizeof self - 1);
  std::string dir = ".";
  if (n > 0) {
    self[n] = 0;
    dir = self;
    dir = dir.substr(0, dir.rfind('/'));
  }
  const std::string path = dir + "/libgpumon_probe.so";
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    *err = std::string("dlopen ") + path + ": " + dlerror();
    return false;
  }
  auto* abi = reinterpret_cast<int (*)()>(dlsym(h, "gpumon_probe_abi_version"));
  g_probe.count = reinterpret_cast<int (*)()>(dlsym(h, "gpumon_probe_device_count"));
  g_probe.create = reinterpret_cast<gpumon_probe* (*)(int, int, int, int, char*, size_t)>(dlsym(h, "gpumon_probe_create"));
  g_probe.launch = reinterpret_cast<int (*)(gpumon_probe*)>(dlsym(h, "gpumon_probe_launch"));
  g_probe.wait = reinterpret_cast<int (*)(gpumon_probe*, int, double, gpumon_probe_result_t*)>(dlsym(h, "gpumon_probe_wait"));
  g_probe.destroy = reinterpret_cast<void (*)(gpumon_probe*)>(dlsym(h, "gpumon_probe_destroy"));
  g_probe.pci = reinterpret_cast<size_t (*)(int, char*, size_t)>(dlsym(h, "gpumon_probe_device_pci"));
  if (!abi || !g_probe.count || !g_probe.create || !g_probe.launch || !g_probe.wait || !g_probe.destroy) {
    *err = path + ": missing symbols";
    return false;
  }
  if (abi() != GPUMON_ONDEVICE_ABI) {
    *err = path + ": plugin ABI mismatch";
    return false;
  }
  g_probe.h = h;  // stays loaded for the life of the helper (HIP keeps its threads)
  return true;
}

gpumon_probe* probe_handle_at(int id) {
  if (id < 0 || id >= static_cast<int>(g_probe.handles.size())) return nullptr;
  return g_probe.handles[id];
}
gpumon_probe* probe_handle(const std::vector<int>& a) { return a.empty() ? nullptr : probe_handle_at(a[0]); }

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

}  // namespace

int main(int argc, char** argv) {
  prctl(PR_SET_PDEATHSIG, SIGKILL);
  // Parent already gone before PDEATHSIG was armed: the exporter passes its pid (a getppid() == 1
  // test is always true when the exporter is PID 1 itself, and misses reparenting to a subreaper).
  long parent = 0;
  for (int i = 1; i < argc; ++i)
    if (!strncmp(argv[i], "--parent-pid=", 13)) parent = strtol(argv[i] + 13, nullptr, 10);
  if (parent > 0 ? getppid() != static_cast<pid_t>(parent) : getppid() == 1) return 0;
  signal(SIGPIPE, SIG_IGN);
  char err[512];
  for (;;) {
    gpumon_pmc_req_t q;
    if (!read_full(0, &q, sizeof q) || q.magic != GPUMON_PMC_PROTO_MAGIC) return 0;
    if (q.n_agents > 4096 || q.counters_len > (64u << 10)) return 0;  // corrupt request: exit
    std::vector<int> agents(q.n_agents);
    std::string counters(q.counters_len, '\0');
    if ((q.n_agents && !read_full(0, agents.data(), agents.size() * sizeof(int))) ||
        (q.counters_len && !read_full(0, &counters[0], counters.size())))
      return 0;
    std::vector<std::string> names;
    for (size_t p = 0; p < counters.size();) {
      size_t e = counters.find('\n', p);
      if (e == std::string::npos) e = counters.size();
      if (e > p) names.push_back(counters.substr(p, e - p));
      p = e + 1;
    }
    std::vector<const char*> cn;
    for (const auto& n : names) cn.push_back(n.c_str());
    err[0] = 0;
    bool ok = true;
    switch (q.op) {
      case GPUMON_PMC_OP_INIT: {
        g_pmc_used = true;
        const int n = gpumon_pmc_init(err, sizeof err);
        ok = reply(n, 0, n < 0 ? err : "", nullptr, 0);
        break;
      }
      case GPUMON_PMC_OP_AGENT: {
        gpumon_pmc_agent_t a{};
        const int rc = agents.empty() ? -1 : gpumon_pmc_agent(agents[0], &a);
        ok = reply(rc, 0, "", rc == 0 ? &a : nullptr, rc == 0 ? sizeof a : 0);
        break;
      }
      case GPUMON_PMC_OP_SAMPLE_MANY:
      case GPUMON_PMC_OP_READ_RUNNING: {
        std::vector<char> payload(agents.size() * cn.size() * sizeof(gpumon_pmc_value_t) +
                                  agents.size() * sizeof(int32_t));
        auto* vals = reinterpret_cast<gpumon_pmc_value_t*>(payload.data());
        auto* oks = reinterpret_cast<int32_t*>(payload.data() + agents.size() * cn.size() * sizeof(gpumon_pmc_value_t));
        int32_t started = 0;
        const int rc = q.op == GPUMON_PMC_OP_SAMPLE_MANY
                           ? gpumon_pmc_sample_many(agents.data(), static_cast<int>(agents.size()), cn.data(),
                                                    static_cast<int>(cn.size()), q.window_s, vals, oks, err, sizeof err)
                           : gpumon_pmc_read_running(agents.data(), static_cast<int>(agents.size()), cn.data(),
                                                     static_cast<int>(cn.size()), vals, oks, &started, err, sizeof err);
        ok = rc == 0 ? reply(0, started, "", payload.data(), payload.size()) : reply(rc, 0, err, nullptr, 0);
        break;
      }
      case GPUMON_PMC_OP_STOP_RUNNING:
        gpumon_pmc_stop_running();
        ok = reply(0, 0, "", nullptr, 0);
        break;
      case GPUMON_PMC_OP_QUIT:
        if (g_pmc_used) gpumon_pmc_stop_running();
        for (auto* p : g_probe.handles)
          if (p) g_probe.destroy(p);
        reply(0, 0, "", nullptr, 0);
        return 0;
      case GPUMON_PROBE_OP_COUNT: {
        std::string e;
        ok = probe_lib(&e) ? reply(g_probe.count(), 0, "", nullptr, 0) : reply(-1, 0, e, nullptr, 0);
        break;
      }
      case GPUMON_PROBE_OP_PCI: {
        std::string e;
        char b[64] = {0};
        if (agents.empty() || !probe_lib(&e)) {
          ok = reply(-1, 0, e.empty() ? "bad probe pci request" : e, nullptr, 0);
          break;
        }
        const size_t len = g_probe.pci ? g_probe.pci(agents[0], b, sizeof b) : 0;
        ok = len > 0 ? reply(static_cast<int>(strlen(b)), 0, "", b, strlen(b)) : reply(0, 0, "", nullptr, 0);
        break;
      }
      case GPUMON_PROBE_OP_CREATE: {
        std::string e;
        if (agents.size() < 4 || !probe_lib(&e)) {
          ok = reply(-1, 0, e.empty() ? "bad probe create request" : e, nullptr, 0);
          break;
        }
        gpumon_probe* p = g_probe.create(agents[0], agents[1], agents[2], agents[3], err, sizeof err);
        if (!p) {
          ok = reply(-1, 0, err, nullptr, 0);
          break;
        }
        g_probe.handles.push_back(p);
        ok = reply(static_cast<int>(g_probe.handles.size()) - 1, 0, "", nullptr, 0);
        break;
      }
      case GPUMON_PROBE_OP_LAUNCH: {
        gpumon_probe* p = probe_handle(agents);
        ok = reply(p ? g_probe.launch(p) : -1, 0, "", nullptr, 0);
        break;
      }
      case GPUMON_PROBE_OP_WAIT: {
        gpumon_probe* p = probe_handle(agents);
        gpumon_probe_result_t r{};
        const int got = p && agents.size() >= 2 ? g_probe.wait(p, agents[1], q.window_s, &r) : 0;
        ok = reply(got, 0, "", got == 1 ? &r : nullptr, got == 1 ? sizeof r : 0);
        break;
      }
      case GPUMON_PROBE_OP_CYCLE: {
        const size_t n = agents.size() / 2;
        std::vector<gpumon_probe_cycle_t> res(n);
        for (size_t k = 0; k < n; ++k) {
          res[k].pending = agents[2 * k + 1];
          res[k].got = 0;
          gpumon_probe* p = probe_handle_at(agents[2 * k]);
          if (p && res[k].pending < 0) res[k].pending = g_probe.launch(p);
        }
        const double t_end = now_s() + q.window_s;
        for (size_t k = 0; k < n; ++k) {
          gpumon_probe* p = probe_handle_at(agents[2 * k]);
          if (!p || res[k].pending < 0) continue;
          if (g_probe.wait(p, res[k].pending, std::max(0.0, t_end - now_s()), &res[k].result) == 1) {
            res[k].got = 1;
            res[k].pending = -1;
          }
        }
        ok = reply(static_cast<int>(n), 0, "", res.data(), res.size() * sizeof(gpumon_probe_cycle_t));
        break;
      }
      case GPUMON_PROBE_OP_DESTROY: {
        gpumon_probe* p = probe_handle(agents);
        if (p) {
          g_probe.destroy(p);
          g_probe.handles[agents[0]] = nullptr;
        }
        ok = reply(0, 0, "", nullptr, 0);
        break;
      }
      default:
        ok = reply(-1, 0, "unknown op", nullptr, 0);
    }
    if (!ok) return 0;
  }
}
