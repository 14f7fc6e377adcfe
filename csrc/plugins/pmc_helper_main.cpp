// bin/gpumon-pmc-helper: owns the rocprofiler-sdk device counting contexts for the exporter
// (protocol and rationale: pmc_helper_proto.h). Reads requests on fd 0, answers on fd 1, links
// lib/libgpumon_pmc.so (rpath $ORIGIN/../lib). Exits on EOF, on QUIT, and with its parent
// (PR_SET_PDEATHSIG SIGKILL: a frozen helper cannot act on SIGTERM).
#include <sys/prctl.h>
#include <unistd.h>

#include <cerrno>
#include <csignal>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ondevice_abi.h"
#include "pmc_helper_proto.h"

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

}  // namespace

int main() {
  prctl(PR_SET_PDEATHSIG, SIGKILL);
  if (getppid() == 1) return 0;  // parent already gone
  signal(SIGPIPE, SIG_IGN);
  char err[512];
  for (;;) {
    gpumon_pmc_req_t q;
    if (!read_full(0, &q, sizeof q) || q.magic != GPUMON_PMC_PROTO_MAGIC) return 0;
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
        gpumon_pmc_stop_running();
        reply(0, 0, "", nullptr, 0);
        return 0;
      default:
        ok = reply(-1, 0, "unknown op", nullptr, 0);
    }
    if (!ok) return 0;
  }
}
