// On-device samplers (PMC device counting + K1 probe) for the native exporter; see ondevice.h.
#include "ondevice.h"

#include <dlfcn.h>
#include <fcntl.h>
#include <poll.h>
#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

#include "../plugins/ondevice_abi.h"
#include "../plugins/ondevice_helper_proto.h"
#include "common.h"
#include "exporter.h"

extern char** environ;

namespace gpumon {

// ---------------------------------------------------------------------------------------------
// plugin loading

struct OnDevice::Plugin {
  void* h = nullptr;
  std::string path;
  // pmc
  int (*pmc_abi)() = nullptr;
  int (*pmc_init)(char*, size_t) = nullptr;
  int (*pmc_agent)(int, gpumon_pmc_agent_t*) = nullptr;
  int (*pmc_sample_many)(const int*, int, const char* const*, int, double, gpumon_pmc_value_t*, int32_t*, char*,
                         size_t) = nullptr;
  // continuous counting (optional symbols)
  int (*pmc_read_running)(const int*, int, const char* const*, int, gpumon_pmc_value_t*, int32_t*, int32_t*, char*,
                          size_t) = nullptr;
  void (*pmc_stop_running)() = nullptr;
  // probe
  int (*probe_abi)() = nullptr;
  int (*probe_count)() = nullptr;
  gpumon_probe* (*probe_create)(int, int, int, int, char*, size_t) = nullptr;
  int (*probe_launch)(gpumon_probe*) = nullptr;
  int (*probe_wait)(gpumon_probe*, int, double, gpumon_probe_result_t*) = nullptr;
  void (*probe_destroy)(gpumon_probe*) = nullptr;
  size_t (*probe_pci)(int, char*, size_t) = nullptr;  // optional: HIP ordinal -> PCI address
  // optional: launch where pending[k] < 0, then wait for every pending launch, in one call
  // (the helper process: one awake period, so the host-observed latency is the GPU's, not IPC's)
  bool (*probe_cycle)(gpumon_probe* const*, int, double, int*, int*, gpumon_probe_result_t*) = nullptr;

  // Plugins stay loaded for the life of the process: rocprofiler keeps the tool's callbacks and
  // the HIP runtime keeps its threads, so dlclose() would leave dangling code pointers.
  ~Plugin() = default;
};

namespace {

template <class F>
bool sym(void* h, const char* name, F* out, std::string* missing) {
  *out = reinterpret_cast<F>(dlsym(h, name));
  if (!*out) *missing += std::string(missing->empty() ? "" : ",") + name;
  return *out != nullptr;
}

std::unique_ptr<OnDevice::Plugin> load_plugin(const std::string& dir, const char* file, bool pmc, std::string* err) {
  auto p = std::make_unique<OnDevice::Plugin>();
  p->path = dir + "/" + file;
  // gpumon._pmc links the same file (rpath $ORIGIN/../lib); the loader matches it by inode, so a
  // process using both holds ONE copy and one rocprofiler tool registration. RTLD_LOCAL keeps a
  // fake plugin (tests) from interposing on a real one loaded later.
  p->h = dlopen(p->path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!p->h) {
    *err = std::string("dlopen ") + p->path + ": " + dlerror();
    return nullptr;
  }
  std::string missing;
  if (pmc) {
    sym(p->h, "gpumon_pmc_abi_version", &p->pmc_abi, &missing);
    sym(p->h, "gpumon_pmc_init", &p->pmc_init, &missing);
    sym(p->h, "gpumon_pmc_agent", &p->pmc_agent, &missing);
    sym(p->h, "gpumon_pmc_sample_many", &p->pmc_sample_many, &missing);
    std::string optional;  // continuous counting: absent -> window mode
    sym(p->h, "gpumon_pmc_read_running", &p->pmc_read_running, &optional);
    sym(p->h, "gpumon_pmc_stop_running", &p->pmc_stop_running, &optional);
  } else {
    sym(p->h, "gpumon_probe_abi_version", &p->probe_abi, &missing);
    sym(p->h, "gpumon_probe_device_count", &p->probe_count, &missing);
    sym(p->h, "gpumon_probe_create", &p->probe_create, &missing);
    sym(p->h, "gpumon_probe_launch", &p->probe_launch, &missing);
    sym(p->h, "gpumon_probe_wait", &p->probe_wait, &missing);
    sym(p->h, "gpumon_probe_destroy", &p->probe_destroy, &missing);
    std::string optional;  // absent -> devices paired by hip_id
    sym(p->h, "gpumon_probe_device_pci", &p->probe_pci, &optional);
  }
  if (!missing.empty()) {
    *err = p->path + ": missing symbols " + missing;
    return nullptr;
  }
  const int abi = pmc ? p->pmc_abi() : p->probe_abi();
  if (abi != GPUMON_ONDEVICE_ABI) {
    *err = p->path + ": plugin ABI " + std::to_string(abi) + " != " + std::to_string(GPUMON_ONDEVICE_ABI);
    return nullptr;
  }
  return p;
}

// ---------------------------------------------------------------------------------------------
// PMC helper process (ondevice_helper_proto.h): the device counting contexts live in
// <plugin dir>/gpumon-ondevice-helper, which this process freezes (SIGSTOP) between requests. The
// functions below have the plugin ABI's signatures, so OnDevice drives the helper through the same
// function table as an in-process plugin. One helper per process.
struct HelperProc {
  std::mutex mu;
  pid_t pid = -1;
  int to = -1, from = -1;  // request pipe (write end), response pipe (read end)
  bool frozen = false;
  std::string path;
};
HelperProc g_helper;

bool io_full(int fd, void* p, size_t n, bool wr, int64_t deadline_ns) {
  auto* b = static_cast<char*>(p);
  while (n) {
    pollfd pf{fd, static_cast<short>(wr ? POLLOUT : POLLIN), 0};
    const int64_t left_ms = (deadline_ns - mono_ns()) / 1000000;
    if (left_ms <= 0 || ::poll(&pf, 1, static_cast<int>(left_ms)) <= 0) return false;
    const ssize_t r = wr ? ::write(fd, b, n) : ::read(fd, b, n);
    if (r < 0 && (errno == EINTR || errno == EAGAIN)) continue;
    if (r <= 0) return false;
    b += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

void helper_kill_locked() {
  if (g_helper.pid > 0) {
    ::kill(g_helper.pid, SIGKILL);  // frozen or hung: SIGKILL works on a stopped process
    int st = 0;
    ::waitpid(g_helper.pid, &st, 0);
  }
  if (g_helper.to >= 0) ::close(g_helper.to);
  if (g_helper.from >= 0) ::close(g_helper.from);
  g_helper.pid = -1;
  g_helper.to = g_helper.from = -1;
  g_helper.frozen = false;
}

// PR_SET_PDEATHSIG (the helper's tie to the exporter) fires when the THREAD that spawned it exits,
// not the process: spawns run on one thread that lives as long as the process, whichever thread
// called start() (a Python caller's worker thread may come and go).
int spawn_on_keeper(const std::function<int()>& job) {
  struct Keeper {
    std::mutex mu;
    std::condition_variable cv;
    const std::function<int()>* job = nullptr;
    int rc = 0;
    bool done = false;
  };
  static Keeper* k = [] {
    auto* kp = new Keeper;  // never freed: the detached thread may still wait on it at exit
    std::thread([kp] {
      set_thread_name("gpumon-spawner");
      std::unique_lock<std::mutex> lk(kp->mu);
      for (;;) {
        kp->cv.wait(lk, [kp] { return kp->job != nullptr; });
        kp->rc = (*kp->job)();
        kp->job = nullptr;
        kp->done = true;
        kp->cv.notify_all();
      }
    }).detach();
    return kp;
  }();
  static std::mutex one;  // one spawn at a time
  std::lock_guard<std::mutex> g(one);
  std::unique_lock<std::mutex> lk(k->mu);
  k->done = false;
  k->job = &job;
  k->cv.notify_all();
  k->cv.wait(lk, [] { return k->done; });
  return k->rc;
}

bool helper_spawn(const std::string& path, std::string* err) {
  std::lock_guard<std::mutex> g(g_helper.mu);
  if (g_helper.pid > 0) return true;
  if (::access(path.c_str(), X_OK) != 0) {
    *err = "on-device helper " + path + " not found / not executable";
    return false;
  }
  int req[2], resp[2];
  if (::pipe2(req, O_CLOEXEC) != 0) {
    *err = std::string("pipe: ") + strerror(errno);
    return false;
  }
  if (::pipe2(resp, O_CLOEXEC) != 0) {
    ::close(req[0]);
    ::close(req[1]);
    *err = std::string("pipe: ") + strerror(errno);
    return false;
  }
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, req[0], 0);
  posix_spawn_file_actions_adddup2(&fa, resp[1], 1);
  // a clean signal state for the child: the exporter may block SIGTERM / SIGINT for its own
  // signal handling, and a signal mask survives exec
  posix_spawnattr_t sa;
  posix_spawnattr_init(&sa);
  sigset_t none, dflt;
  sigemptyset(&none);
  sigemptyset(&dflt);
  for (int s : {SIGTERM, SIGINT, SIGHUP, SIGPIPE}) sigaddset(&dflt, s);
  posix_spawnattr_setsigmask(&sa, &none);
  posix_spawnattr_setsigdefault(&sa, &dflt);
  posix_spawnattr_setflags(&sa, POSIX_SPAWN_SETSIGMASK | POSIX_SPAWN_SETSIGDEF);
  // the helper checks its parent against this pid, not against 1: the exporter may itself be
  // PID 1 (ENTRYPOINT without hostPID), and an orphan under hostPID goes to a subreaper, not 1
  std::string parent = "--parent-pid=" + std::to_string(::getpid());
  char* argv[] = {const_cast<char*>(path.c_str()), const_cast<char*>(parent.c_str()), nullptr};
  pid_t pid = -1;
  const int rc = spawn_on_keeper([&] { return posix_spawn(&pid, path.c_str(), &fa, &sa, argv, environ); });
  posix_spawnattr_destroy(&sa);
  posix_spawn_file_actions_destroy(&fa);
  ::close(req[0]);
  ::close(resp[1]);
  if (rc != 0) {
    ::close(req[1]);
    ::close(resp[0]);
    *err = "posix_spawn " + path + ": " + strerror(rc);
    return false;
  }
  g_helper.pid = pid;
  g_helper.to = req[1];
  g_helper.from = resp[0];
  g_helper.frozen = false;
  g_helper.path = path;
  return true;
}

bool helper_alive() {
  std::lock_guard<std::mutex> g(g_helper.mu);
  return g_helper.pid > 0;
}

// The helper's CPU seconds and resident bytes from /proc (it is part of the pod's footprint: the
// exporter's own process_* series do not include it). False when it is not running.
bool helper_usage(double* cpu_s, double* rss_bytes) {
  pid_t pid;
  {
    std::lock_guard<std::mutex> g(g_helper.mu);
    pid = g_helper.pid;
  }
  if (pid <= 0) return false;
  char buf[1024];
  FILE* f = fopen(("/proc/" + std::to_string(pid) + "/stat").c_str(), "r");
  if (!f) return false;
  const size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* p = strrchr(buf, ')');
  if (!p) return false;
  // fields after "(comm)": state(3) ... utime(14) stime(15) ... rss(24, pages)
  unsigned long long v[22] = {0};
  int k = 0;
  for (const char* q = p + 2; *q && k < 22; ++k) {
    while (*q == ' ') ++q;
    if (k > 0) v[k] = strtoull(q, nullptr, 10);
    while (*q && *q != ' ') ++q;
  }
  const double hz = static_cast<double>(sysconf(_SC_CLK_TCK));
  *cpu_s = (v[11] + v[12]) / hz;  // utime, stime
  *rss_bytes = static_cast<double>(v[21]) * static_cast<double>(sysconf(_SC_PAGESIZE));
  return true;
}

// One request / response; the helper runs only for the duration of the call.
int helper_call(uint32_t op, const int* agents, int n_agents, const char* const* counters, int n_counters,
                double window_s, std::vector<char>* payload, int32_t* started, std::string* err) {
  std::lock_guard<std::mutex> g(g_helper.mu);
  if (g_helper.pid <= 0) {
    *err = "on-device helper not running";
    return -1;
  }
  if (g_helper.frozen) {
    ::kill(g_helper.pid, SIGCONT);
    g_helper.frozen = false;
  }
  std::string names;
  for (int c = 0; c < n_counters; ++c) names += std::string(counters[c]) + "\n";
  gpumon_pmc_req_t q{GPUMON_PMC_PROTO_MAGIC, op, static_cast<uint32_t>(std::max(0, n_agents)),
                     static_cast<uint32_t>(names.size()), window_s};
  // init brings HSA + rocprofiler up, and the first probe op HIP (seconds on a fresh node, more
  // while the runtime pages in); a read or a probe cycle takes milliseconds plus its own window
  const bool slow = op == GPUMON_PMC_OP_INIT || op == GPUMON_PROBE_OP_COUNT || op == GPUMON_PROBE_OP_CREATE;
  const int64_t deadline = mono_ns() + static_cast<int64_t>((slow ? 60.0 : 10.0 + window_s) * 1e9);
  gpumon_pmc_resp_t h{};
  std::string e;
  bool ok = io_full(g_helper.to, &q, sizeof q, true, deadline) &&
            (n_agents <= 0 || io_full(g_helper.to, const_cast<int*>(agents), sizeof(int) * n_agents, true, deadline)) &&
            (names.empty() || io_full(g_helper.to, &names[0], names.size(), true, deadline)) &&
            io_full(g_helper.from, &h, sizeof h, false, deadline) && h.magic == GPUMON_PMC_PROTO_MAGIC &&
            h.err_len <= (64u << 10) && h.payload_len <= (16u << 20);  // a corrupt header is a dead helper
  if (ok && h.err_len) {
    e.resize(h.err_len);
    ok = io_full(g_helper.from, &e[0], e.size(), false, deadline);
  }
  if (ok) {
    payload->resize(h.payload_len);
    ok = h.payload_len == 0 || io_full(g_helper.from, payload->data(), payload->size(), false, deadline);
  }
  if (!ok) {
    *err = "on-device helper " + g_helper.path + " died or timed out";
    helper_kill_locked();  // the next start spawns a fresh one
    return -1;
  }
  if (op != GPUMON_PMC_OP_QUIT && ::kill(g_helper.pid, SIGSTOP) == 0) g_helper.frozen = true;
  if (started) *started = h.started;
  *err = e;
  return h.rc;
}

int h_abi() { return GPUMON_ONDEVICE_ABI; }
int h_init(char* err, size_t n) {
  std::vector<char> p;
  std::string e;
  const int rc = helper_call(GPUMON_PMC_OP_INIT, nullptr, 0, nullptr, 0, 0, &p, nullptr, &e);
  if (rc < 0 && err && n) snprintf(err, n, "%s", e.c_str());
  return rc;
}
int h_agent(int agent, gpumon_pmc_agent_t* out) {
  std::vector<char> p;
  std::string e;
  if (helper_call(GPUMON_PMC_OP_AGENT, &agent, 1, nullptr, 0, 0, &p, nullptr, &e) != 0 ||
      p.size() != sizeof(gpumon_pmc_agent_t))
    return -1;
  memcpy(out, p.data(), sizeof *out);
  return 0;
}
int h_values(uint32_t op, const int* agents, int n_agents, const char* const* counters, int n_counters,
             double window_s, gpumon_pmc_value_t* out, int32_t* ok, int32_t* started, char* err, size_t errlen) {
  std::vector<char> p;
  std::string e;
  const int rc = helper_call(op, agents, n_agents, counters, n_counters, window_s, &p, started, &e);
  const size_t nv = static_cast<size_t>(n_agents) * n_counters;
  if (rc != 0 || p.size() != nv * sizeof(gpumon_pmc_value_t) + n_agents * sizeof(int32_t)) {
    if (err && errlen) snprintf(err, errlen, "%s", e.empty() ? "on-device helper: bad response" : e.c_str());
    return rc != 0 ? rc : -1;
  }
  memcpy(out, p.data(), nv * sizeof(gpumon_pmc_value_t));
  memcpy(ok, p.data() + nv * sizeof(gpumon_pmc_value_t), n_agents * sizeof(int32_t));
  return 0;
}
int h_sample_many(const int* a, int na, const char* const* c, int nc, double w, gpumon_pmc_value_t* out, int32_t* ok,
                  char* err, size_t errlen) {
  return h_values(GPUMON_PMC_OP_SAMPLE_MANY, a, na, c, nc, w, out, ok, nullptr, err, errlen);
}
int h_read_running(const int* a, int na, const char* const* c, int nc, gpumon_pmc_value_t* out, int32_t* ok,
                   int32_t* started, char* err, size_t errlen) {
  return h_values(GPUMON_PMC_OP_READ_RUNNING, a, na, c, nc, 0, out, ok, started, err, errlen);
}
void h_stop_running() {
  std::vector<char> p;
  std::string e;
  helper_call(GPUMON_PMC_OP_STOP_RUNNING, nullptr, 0, nullptr, 0, 0, &p, nullptr, &e);
}

// K1 probe through the helper: a handle is the helper's probe id + 1 disguised as the pointer type
int h_probe_count() {
  std::vector<char> p;
  std::string e;
  const int rc = helper_call(GPUMON_PROBE_OP_COUNT, nullptr, 0, nullptr, 0, 0, &p, nullptr, &e);
  if (rc < 0) GPUMON_LOG(LogLevel::kWarn, "ondevice", "probe device count (helper): " + e);
  return rc < 0 ? 0 : rc;
}
gpumon_probe* h_probe_create(int dev, int blocks, int slots, int spin, char* err, size_t errlen) {
  const int a[4] = {dev, blocks, slots, spin};
  std::vector<char> p;
  std::string e;
  const int rc = helper_call(GPUMON_PROBE_OP_CREATE, a, 4, nullptr, 0, 0, &p, nullptr, &e);
  if (rc < 0) {
    if (err && errlen) snprintf(err, errlen, "%s", e.c_str());
    return nullptr;
  }
  return reinterpret_cast<gpumon_probe*>(static_cast<intptr_t>(rc) + 1);
}
int h_probe_id(gpumon_probe* h) { return static_cast<int>(reinterpret_cast<intptr_t>(h) - 1); }
int h_probe_launch(gpumon_probe* h) {
  const int a[1] = {h_probe_id(h)};
  std::vector<char> p;
  std::string e;
  return helper_call(GPUMON_PROBE_OP_LAUNCH, a, 1, nullptr, 0, 0, &p, nullptr, &e);
}
int h_probe_wait(gpumon_probe* h, int slot, double timeout_s, gpumon_probe_result_t* out) {
  const int a[2] = {h_probe_id(h), slot};
  std::vector<char> p;
  std::string e;
  const int rc = helper_call(GPUMON_PROBE_OP_WAIT, a, 2, nullptr, 0, timeout_s, &p, nullptr, &e);
  if (rc != 1 || p.size() != sizeof *out) return 0;
  memcpy(out, p.data(), sizeof *out);
  return 1;
}
size_t h_probe_pci(int dev, char* buf, size_t len) {
  const int a[1] = {dev};
  std::vector<char> p;
  std::string e;
  const int rc = helper_call(GPUMON_PROBE_OP_PCI, a, 1, nullptr, 0, 0, &p, nullptr, &e);
  if (rc <= 0 || p.empty() || !buf || !len) return 0;
  const size_t n = std::min(p.size(), len - 1);
  memcpy(buf, p.data(), n);
  buf[n] = 0;
  return n + 1;
}
void h_probe_destroy(gpumon_probe* h) {
  const int a[1] = {h_probe_id(h)};
  std::vector<char> p;
  std::string e;
  helper_call(GPUMON_PROBE_OP_DESTROY, a, 1, nullptr, 0, 0, &p, nullptr, &e);
}

bool h_probe_cycle(gpumon_probe* const* hs, int n, double timeout_s, int* pending, int* got,
                   gpumon_probe_result_t* out) {
  std::vector<int> a(2 * static_cast<size_t>(n));
  for (int k = 0; k < n; ++k) {
    a[2 * k] = h_probe_id(hs[k]);
    a[2 * k + 1] = pending[k];
  }
  std::vector<char> p;
  std::string e;
  const int rc = helper_call(GPUMON_PROBE_OP_CYCLE, a.data(), 2 * n, nullptr, 0, timeout_s, &p, nullptr, &e);
  if (rc != n || p.size() != n * sizeof(gpumon_probe_cycle_t)) {
    for (int k = 0; k < n; ++k) got[k] = 0;  // pending unknown: keep the caller's (a later wait times out)
    return false;
  }
  for (int k = 0; k < n; ++k) {
    gpumon_probe_cycle_t c;
    memcpy(&c, p.data() + k * sizeof c, sizeof c);
    pending[k] = c.pending;
    got[k] = c.got;
    if (c.got) out[k] = c.result;
  }
  return true;
}

void helper_shutdown() {
  {
    std::vector<char> p;
    std::string e;
    helper_call(GPUMON_PMC_OP_QUIT, nullptr, 0, nullptr, 0, 0, &p, nullptr, &e);
  }
  std::lock_guard<std::mutex> g(g_helper.mu);
  if (g_helper.pid > 0) {
    const int64_t until = mono_ns() + 2'000'000'000;
    int st = 0;
    while (mono_ns() < until && ::waitpid(g_helper.pid, &st, WNOHANG) == 0)
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    if (::waitpid(g_helper.pid, &st, WNOHANG) == 0) helper_kill_locked();
    else {
      g_helper.pid = -1;
      helper_kill_locked();  // closes the pipes
    }
  }
}

ExtraSeries xs(const char* name, const char* help, int dev, double v, const char* type = "gauge") {
  ExtraSeries s;
  s.name = name;
  s.help = help;
  s.type = type;
  s.dev = dev;
  s.value = v;
  return s;
}

}  // namespace

int ondevice_helper_pid() {
  std::lock_guard<std::mutex> g(g_helper.mu);
  return g_helper.pid;
}

std::string default_plugin_dir() {
  if (const char* e = getenv("GPUMON_PLUGIN_DIR"); e && *e) return e;
  Dl_info info{};
  // The object holding this function: bin/gpumon-exporter or gpumon/_core*.so; both sit one level
  // below the tree root, next to lib/.
  if (dladdr(reinterpret_cast<void*>(&default_plugin_dir), &info) && info.dli_fname) {
    std::string f = info.dli_fname;
    if (f.find('/') == std::string::npos) {
      char buf[4096];
      ssize_t n = readlink("/proc/self/exe", buf, sizeof buf - 1);
      if (n > 0) f.assign(buf, static_cast<size_t>(n));
    }
    auto slash = f.rfind('/');
    std::string dir = slash == std::string::npos ? "." : f.substr(0, slash);
    return dir + "/../lib";
  }
  return "lib";
}

// ---------------------------------------------------------------------------------------------
// derivation (mirrors tests/oracles/ops/pmc.py derive())

PmcDerived pmc_derive(const std::map<std::string, PmcReduced>& raw, const PmcAgentInfo& agent, double window_s) {
  PmcDerived d;
  if (window_s > 0) {
    static const std::string kMops = "SQ_INSTS_VALU_MFMA_MOPS_";
    for (const auto& [name, v] : raw) {  // std::map: sorted by counter name
      if (name.compare(0, kMops.size(), kMops) != 0) continue;
      std::string dt = name.substr(kMops.size());
      for (auto& c : dt) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
      d.mfma_tflops.emplace_back(dt, 512.0 * v.sum / window_s / 1e12);
    }
  }
  auto get = [&](const char* k) -> const PmcReduced* {
    auto it = raw.find(k);
    return it == raw.end() ? nullptr : &it->second;
  };
  const PmcReduced* gui_r = get("GRBM_GUI_ACTIVE");
  const double gui = gui_r ? gui_r->max : 0.0;
  const double simds = agent.simd_count ? agent.simd_count : agent.cu_count * 4.0;
  const double cus = agent.cu_count;
  const double waves = agent.max_waves_per_cu ? agent.max_waves_per_cu : 32.0;
  if (gui > 0 && simds > 0) {
    if (const PmcReduced* m = get("SQ_VALU_MFMA_BUSY_CYCLES")) {
      d.mfma_busy = std::min(100.0, 100.0 * m->sum / (gui * simds));
      if (m->by_xcc.size() > 1) {
        const double per = simds / m->by_xcc.size();
        for (double v : m->by_xcc) d.xcd_mfma_busy.push_back(std::min(100.0, 100.0 * v / (gui * per)));
      }
    }
  }
  if (gui > 0 && cus > 0)
    if (const PmcReduced* w = get("SQ_WAVE_CYCLES")) d.occupancy = std::min(100.0, 400.0 * w->sum / gui / cus / waves);
  if (const PmcReduced* c = get("GRBM_COUNT"); c && c->max > 0) d.gui_active = std::min(100.0, 100.0 * gui / c->max);
  return d;
}

// ---------------------------------------------------------------------------------------------

OnDevice::OnDevice(Exporter* ex, OnDeviceConfig cfg) : ex_(ex), cfg_(std::move(cfg)) {
  cfg_.pmc_window_s = std::max(0.001, std::min(cfg_.pmc_window_s, cfg_.pmc_every_s * 0.5));
  cfg_.pmc_every_s = std::max(0.01, cfg_.pmc_every_s);
  cfg_.probe_timeout_s = std::min(cfg_.probe_timeout_s, cfg_.probe_every_s);
}

OnDevice::~OnDevice() { stop(); }

bool OnDevice::start(std::string* err) {
  if (stopped_) {
    *err = "on-device samplers already stopped";
    return false;
  }
  const std::string dir = cfg_.plugin_dir.empty() ? default_plugin_dir() : cfg_.plugin_dir;
  char ebuf[512] = {0};
  if (cfg_.ondevice_isolate && (cfg_.pmc || cfg_.probe)) {
    // device counting contexts and the probe in one helper process, frozen between requests
    // (ondevice_helper_proto.h): this process never loads HIP, HSA or rocprofiler-sdk
    helper_path_ = dir + "/gpumon-ondevice-helper";
    if (!helper_spawn(helper_path_, err)) return false;
    helper_ = true;
    helper_spawned_ns_ = mono_ns();
  }
  if (cfg_.pmc) {
    if (cfg_.ondevice_isolate) {
      pmc_lib_ = std::make_unique<Plugin>();
      pmc_lib_->path = dir + "/gpumon-ondevice-helper";
      pmc_lib_->pmc_abi = &h_abi;
      pmc_lib_->pmc_init = &h_init;
      pmc_lib_->pmc_agent = &h_agent;
      pmc_lib_->pmc_sample_many = &h_sample_many;
      pmc_lib_->pmc_read_running = &h_read_running;
      pmc_lib_->pmc_stop_running = &h_stop_running;
    } else {
      pmc_lib_ = load_plugin(dir, "libgpumon_pmc.so", true, err);
    }
    if (!pmc_lib_) return false;
    const int n = pmc_lib_->pmc_init(ebuf, sizeof ebuf);
    if (n < 0) {
      *err = std::string("pmc init: ") + ebuf;
      pmc_lib_.reset();
      if (helper_) helper_shutdown();
      return false;
    }
    gpumon_pmc_agent_t a{};
    for (int i = 0; i < n && pmc_lib_->pmc_agent(i, &a) == 0; ++i) {
      PmcAgentInfo ai;
      ai.cu_count = a.cu_count;
      ai.simd_count = a.simd_count;
      ai.num_xcc = a.num_xcc;
      ai.max_waves_per_cu = a.max_waves_per_cu;
      ai.drm_render_minor = a.drm_render_minor;
      agents_.push_back(ai);
    }
    map_pmc_agents();
    pmc_continuous_ = cfg_.pmc_mode != "window" && pmc_lib_->pmc_read_running && pmc_lib_->pmc_stop_running;
    GPUMON_LOG(LogLevel::kInfo, "ondevice",
               "pmc plugin " + pmc_lib_->path + " agents=" + std::to_string(agents_.size()) +
                   " mapped=" + std::to_string(pmc_map_.size()) +
                   (pmc_continuous_ ? " mode=continuous" : " mode=window"));
  }
  if (cfg_.probe) {
    if (cfg_.ondevice_isolate) {
      probe_lib_ = std::make_unique<Plugin>();
      probe_lib_->path = dir + "/gpumon-ondevice-helper";
      probe_lib_->probe_abi = &h_abi;
      probe_lib_->probe_count = &h_probe_count;
      probe_lib_->probe_create = &h_probe_create;
      probe_lib_->probe_launch = &h_probe_launch;
      probe_lib_->probe_wait = &h_probe_wait;
      probe_lib_->probe_destroy = &h_probe_destroy;
      probe_lib_->probe_cycle = &h_probe_cycle;
      probe_lib_->probe_pci = &h_probe_pci;
    } else {
      probe_lib_ = load_plugin(dir, "libgpumon_probe.so", false, err);
    }
    if (!probe_lib_) {
      pmc_lib_.reset();
      if (helper_) helper_shutdown();
      return false;
    }
    if (!create_probes(err)) {
      if (helper_) helper_shutdown();
      return false;
    }
    GPUMON_LOG(LogLevel::kInfo, "ondevice",
               "probe plugin " + probe_lib_->path + " devices=" + std::to_string(probes_.size()) +
                   (probes_.empty() ? " (device list not known yet: created on the first step that has it)" : ""));
  }
  if (helper_) export_helper();
  running_ = true;
  if (pmc_lib_) pmc_th_ = std::thread([this] {
    set_thread_name("gpumon-pmc");
    pmc_loop();
  });
  if (probe_lib_) probe_th_ = std::thread([this] {
    set_thread_name("gpumon-probe");
    probe_loop();
  });
  return true;
}

void OnDevice::stop() {
  // idempotent: the destructor calls it again, possibly during interpreter teardown, and must not
  // touch the exporter a second time
  if (stopped_.exchange(true)) return;
  if (running_.exchange(false)) {
    std::lock_guard<std::mutex> g(wait_mu_);  // no lost wake-up between the check and the wait
    wait_cv_.notify_all();
  }
  if (pmc_th_.joinable()) pmc_th_.join();
  if (probe_th_.joinable()) probe_th_.join();
  if (pmc_lib_ && pmc_continuous_) pmc_lib_->pmc_stop_running();  // release the device counters
  if (probe_lib_) {
    std::lock_guard<std::mutex> g(probe_mu_);
    gpumon_probe_result_t r{};
    for (auto& p : probes_) {
      // drain the in-flight launch before its pinned ring is freed
      if (p.pending >= 0) probe_lib_->probe_wait(static_cast<gpumon_probe*>(p.handle), p.pending, 2.0, &r);
      probe_lib_->probe_destroy(static_cast<gpumon_probe*>(p.handle));
    }
    probes_.clear();
    ex_->set_extra("probe", {});
  }
  if (helper_) {
    helper_shutdown();  // after the probes' rings are drained and freed
    ex_->set_extra("ondevice_helper", {});
  }
  if (pmc_lib_) {
    ex_->set_extra("pmc", {});
    ex_->set_device_mfma_util({});
  }
}

bool OnDevice::step() {
  if (pmc_lib_) {
    pmc_step();
    // continuous mode: a first read only starts the counting; a synchronous step (tests, --once)
    // must produce values, so read again after one window
    bool empty;
    {
      std::lock_guard<std::mutex> g(pmc_mu_);
      empty = pmc_continuous_ && pmc_last_.empty() && pmc_up_;
    }
    if (empty) {
      std::this_thread::sleep_for(std::chrono::duration<double>(cfg_.pmc_window_s));
      pmc_step();
    }
  }
  if (probe_lib_) probe_step();
  return pmc_lib_ || probe_lib_;
}

OnDevice::Stats OnDevice::stats() const {
  Stats s;
  s.pmc_samples = pmc_samples_;
  s.pmc_steps = pmc_steps_;
  s.probe_steps = probe_steps_;
  s.pmc_errors = pmc_errors_;
  s.pmc_resets = pmc_resets_;
  s.pmc_continuous = pmc_continuous_;
  s.probe_done = probe_done_;
  s.probe_timeouts = probe_timeouts_;
  s.pmc_agents = static_cast<int>(agents_.size());
  s.probe_devices = static_cast<int>(probes_.size());
  s.probe_by_bdf = probe_by_bdf_;
  s.helper_restarts = helper_restarts_;
  return s;
}

bool OnDevice::helper_check() {
  if (!helper_) return true;
  std::lock_guard<std::mutex> g(recover_mu_);
  if (helper_alive()) return true;
  const int64_t now = mono_ns();
  if (now < next_respawn_ns_) return false;
  // a helper that keeps dying soon after its start (OOM-killed under a tight memory limit, a
  // broken driver) is retried with exponential backoff: helper_retry_s x 2^streak, at most 64x;
  // one that ran for 10 minutes resets the streak
  if (helper_spawned_ns_ && now - helper_spawned_ns_ > 600'000'000'000ll) respawn_streak_ = 0;
  const double backoff = std::max(0.0, cfg_.helper_retry_s) * static_cast<double>(1 << std::min(respawn_streak_, 6));
  next_respawn_ns_ = now + static_cast<int64_t>(backoff * 1e9);
  respawn_streak_++;
  std::string err;
  if (!helper_spawn(helper_path_, &err)) {
    GPUMON_LOG(LogLevel::kWarn, "ondevice", "on-device helper respawn failed: " + err);
    return false;
  }
  if (pmc_lib_) {  // rocprofiler must register before anything brings HSA up in the new helper
    char ebuf[512] = {0};
    if (pmc_lib_->pmc_init(ebuf, sizeof ebuf) < 0) {
      GPUMON_LOG(LogLevel::kWarn, "ondevice", std::string("on-device helper respawned, pmc init failed: ") + ebuf);
      helper_shutdown();
      return false;
    }
  }
  helper_spawned_ns_ = mono_ns();
  helper_gen_++;  // probe handles of the dead helper are void; the probe sampler recreates them
  helper_restarts_++;
  GPUMON_LOG(LogLevel::kWarn, "ondevice",
             "on-device helper was gone: respawned " + helper_path_ + " (restart " +
                 std::to_string(helper_restarts_.load()) + ")");
  export_helper();
  return true;
}

void OnDevice::export_helper() {
  std::vector<ExtraSeries> out = {
      xs("gpumon_ondevice_helper_restarts_total",
         "Times the on-device helper process (PMC contexts + K1 probe) was found dead and respawned.", -1,
         static_cast<double>(helper_restarts_.load()), "counter")};
  double cpu = 0, rss = 0;
  if (helper_usage(&cpu, &rss)) {
    out.push_back(xs("gpumon_ondevice_helper_cpu_seconds_total",
                     "CPU time of the on-device helper process (part of the pod's footprint; process_* "
                     "series cover the exporter process only).",
                     -1, cpu, "counter"));
    out.push_back(xs("gpumon_ondevice_helper_resident_memory_bytes",
                     "Resident memory of the on-device helper process (its GPU runtimes).", -1, rss));
  }
  // What the enabled samplers should hold (profiles/r3_helper_memory.md, r3_probe_hsa.md): 0.11 GB
  // of runtime plus one fully resident 173 MB context-save block per hardware queue per GPU --
  // device counting alone brings up 2 queues per GPU, the K1 probe alone 2, both together 3 (the
  // runtime's copy queue is shared). The memory alert compares the helper's RSS with this.
  const int blocks = cfg_.pmc && cfg_.probe ? 3 : (cfg_.pmc || cfg_.probe) ? 2 : 0;
  const double gpus = static_cast<double>(ex_->statics().size());
  out.push_back(xs("gpumon_ondevice_helper_memory_model_bytes",
                   "Expected resident memory of the on-device helper for the enabled samplers: 0.11 GB + 173 MB "
                   "per hardware queue per GPU (PMC 2 queues, probe 2, both 3).",
                   -1, 110e6 + gpus * blocks * 173e6));
  ex_->set_extra("ondevice_helper", std::move(out));
}

// ---------------------------------------------------------------------------------------------
// PMC

void OnDevice::map_pmc_agents() {
  pmc_map_.clear();
  for (const auto& s : ex_->statics()) {
    for (size_t ai = 0; ai < agents_.size(); ++ai) {
      if ((s.drm_render >= 0 && s.drm_render == agents_[ai].drm_render_minor) ||
          (s.drm_render < 0 && static_cast<int>(ai) == s.index)) {
        pmc_map_[s.index] = static_cast<int>(ai);
        break;
      }
    }
  }
}

void OnDevice::pmc_step() {
  std::lock_guard<std::mutex> g(pmc_mu_);
  pmc_steps_++;
  if (helper_) export_helper();
  if (!helper_check()) {  // helper gone, respawn not due yet: no values, series withdrawn
    pmc_errors_++;
    pmc_up_ = false;
    pmc_prev_.clear();
    pmc_last_.clear();
    export_pmc();
    return;
  }
  if (pmc_map_.empty()) map_pmc_agents();  // backend came up after start()
  if (pmc_map_.empty()) return;
  std::vector<int> devs, ags;
  for (const auto& kv : pmc_map_) {
    devs.push_back(kv.first);
    ags.push_back(kv.second);
  }
  if (pmc_continuous_) pmc_step_continuous(devs, ags);
  else pmc_step_window(devs, ags);
  export_pmc();
}

namespace {
PmcReduced to_reduced(const gpumon_pmc_value_t& v) {
  PmcReduced r;
  r.sum = v.sum;
  r.max = v.max;
  r.n = v.n;
  r.by_xcc.assign(v.by_xcc, v.by_xcc + std::max(0, std::min<int>(v.n_xcc, GPUMON_PMC_MAX_XCC)));
  return r;
}
}  // namespace

// Wall-time MFMA utilisation: the active-cycle share times the share of WALL time the GPU was
// active. GRBM_COUNT cannot give the latter -- the shader clock drops while idle (2.25 -> 1.58 GHz
// in a 500 ms on / off burst on MI355X), so cycle shares over-weight busy time -- but the
// firmware's gfx activity accumulator is wall-time based: the product tracks event-timed duty
// loads within 3 points, bursts included (profiles/r2_pmc_continuous.md).
void OnDevice::finish_derived(int dev, PmcDerived* d) {
  double act = kNaN;
  std::array<double, kMaxXcc> xcd_act{};
  int n_xcd = 0;
  const auto rates = ex_->rates();
  if (dev >= 0 && dev < static_cast<int>(rates.size()) && rates[dev].valid) {
    act = rates[dev].gfx_activity_avg_pct;
    n_xcd = rates[dev].n_xcd;
    xcd_act = rates[dev].xcd_busy_avg;
  }
  if (!has(act)) act = d->gui_active;  // no firmware activity: the cycle share is the best left
  if (has(d->mfma_busy) && has(act)) d->mfma_util = std::min(100.0, d->mfma_busy * act / 100.0);
  d->xcd_mfma_util.clear();
  for (size_t x = 0; x < d->xcd_mfma_busy.size(); ++x) {
    const double a = static_cast<int>(x) < n_xcd && has(xcd_act[x]) ? xcd_act[x] : act;
    if (has(a)) d->xcd_mfma_util.push_back(std::min(100.0, d->xcd_mfma_busy[x] * a / 100.0));
  }
}

void OnDevice::pmc_step_window(const std::vector<int>& devs, const std::vector<int>& ags) {
  std::vector<const char*> names;
  for (const auto& c : cfg_.pmc_counters) names.push_back(c.c_str());
  std::vector<gpumon_pmc_value_t> vals(devs.size() * names.size());
  std::vector<int32_t> ok(devs.size(), 0);
  char ebuf[512] = {0};
  // every GPU counts over ONE shared window (8 GPUs: one window, not eight)
  const int rc = pmc_lib_->pmc_sample_many(ags.data(), static_cast<int>(ags.size()), names.data(),
                                           static_cast<int>(names.size()), cfg_.pmc_window_s, vals.data(), ok.data(),
                                           ebuf, sizeof ebuf);
  if (rc != 0) {
    pmc_errors_ += devs.size();
    pmc_up_ = false;
    GPUMON_LOG(LogLevel::kWarn, "ondevice", std::string("pmc sample failed: ") + ebuf);
    return;
  }
  pmc_up_ = true;
  for (size_t k = 0; k < devs.size(); ++k) {
    if (!ok[k]) {
      pmc_errors_++;
      continue;
    }
    std::map<std::string, PmcReduced> raw;
    for (size_t c = 0; c < names.size(); ++c)
      if (vals[k * names.size() + c].ok) raw[cfg_.pmc_counters[c]] = to_reduced(vals[k * names.size() + c]);
    PmcDerived d = pmc_derive(raw, agents_[ags[k]], cfg_.pmc_window_s);
    d.span_s = cfg_.pmc_window_s;
    d.coverage = cfg_.pmc_window_s / cfg_.pmc_every_s;
    finish_derived(devs[k], &d);
    pmc_last_[devs[k]] = std::move(d);
    pmc_samples_++;
  }
}

void OnDevice::pmc_step_continuous(const std::vector<int>& devs, const std::vector<int>& ags) {
  std::vector<const char*> names;
  for (const auto& c : cfg_.pmc_counters) names.push_back(c.c_str());
  std::vector<gpumon_pmc_value_t> vals(devs.size() * names.size());
  std::vector<int32_t> ok(devs.size(), 0);
  int32_t started = 0;
  char ebuf[512] = {0};
  const int rc = pmc_lib_->pmc_read_running(ags.data(), static_cast<int>(ags.size()), names.data(),
                                            static_cast<int>(names.size()), vals.data(), ok.data(), &started, ebuf,
                                            sizeof ebuf);
  const int64_t now = mono_ns();
  if (rc != 0) {
    // contexts could not start / be read (another profiler holds the counters?): no values this
    // step, the series withdrawn (never stale values), and the next step tries again from scratch
    pmc_errors_ += devs.size();
    if (pmc_up_) GPUMON_LOG(LogLevel::kWarn, "ondevice", std::string("pmc continuous read failed: ") + ebuf);
    pmc_up_ = false;
    pmc_prev_.clear();
    pmc_last_.clear();
    return;
  }
  pmc_up_ = true;
  const double dt = pmc_prev_ns_ ? (now - pmc_prev_ns_) * 1e-9 : 0.0;
  for (size_t k = 0; k < devs.size(); ++k) {
    if (!ok[k]) {
      pmc_errors_++;
      pmc_prev_.erase(devs[k]);
      pmc_last_.erase(devs[k]);
      continue;
    }
    std::map<std::string, PmcReduced> cur;
    for (size_t c = 0; c < names.size(); ++c)
      if (vals[k * names.size() + c].ok) cur[cfg_.pmc_counters[c]] = to_reduced(vals[k * names.size() + c]);
    auto prev_it = pmc_prev_.find(devs[k]);
    if (!started && prev_it != pmc_prev_.end() && dt > 0) {
      // counts are cumulative since the context start: the interval is the difference
      std::map<std::string, PmcReduced> delta;
      bool reset = false;
      for (const auto& [name, v] : cur) {
        auto p = prev_it->second.find(name);
        if (p == prev_it->second.end()) continue;
        PmcReduced d;
        d.sum = v.sum - p->second.sum;
        d.max = v.max - p->second.max;
        d.n = v.n;
        if (d.sum < 0 || d.max < 0) reset = true;  // restarted underneath us: drop this interval
        d.by_xcc.resize(v.by_xcc.size());
        for (size_t x = 0; x < v.by_xcc.size(); ++x)
          d.by_xcc[x] = v.by_xcc[x] - (x < p->second.by_xcc.size() ? p->second.by_xcc[x] : 0.0);
        delta[name] = std::move(d);
      }
      if (reset) {
        pmc_resets_++;
        pmc_last_.erase(devs[k]);
      } else {
        PmcDerived d = pmc_derive(delta, agents_[ags[k]], dt);
        d.span_s = dt;
        d.coverage = 1.0;
        finish_derived(devs[k], &d);
        pmc_last_[devs[k]] = std::move(d);
        pmc_samples_++;
      }
    }
    pmc_prev_[devs[k]] = std::move(cur);
  }
  pmc_prev_ns_ = now;
}

void OnDevice::export_pmc() {
  std::vector<ExtraSeries> out;
  std::map<int, double> mfma;  // for pod_gpu_mfma_util_percent (exclusive use)
  for (const auto& kv : pmc_last_)
    if (!std::isnan(kv.second.mfma_util)) mfma[kv.first] = kv.second.mfma_util;
  ex_->set_device_mfma_util(std::move(mfma));
  for (const auto& kv : pmc_last_) {
    const int dev = kv.first;
    const PmcDerived& d = kv.second;
    if (!std::isnan(d.mfma_util))
      out.push_back(xs("gpu_mfma_util_percent",
                       "MFMA pipes busy as a share of wall time, in percent: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE "
                       "x SIMDs) x the firmware's wall-time gfx activity over the interval (every process).",
                       dev, d.mfma_util));
    for (size_t x = 0; x < d.xcd_mfma_util.size(); ++x) {
      out.push_back(xs("gpu_xcd_mfma_util_percent", "MFMA pipes busy as a share of wall time per XCD, in percent.", dev,
                       d.xcd_mfma_util[x]));
      out.back().labels.push_back({"xcd", std::to_string(x)});
    }
    if (!std::isnan(d.mfma_busy))
      out.push_back(xs("gpu_mfma_busy_active_percent",
                       "MFMA pipes busy as a share of the GPU's ACTIVE cycles (GRBM_GUI_ACTIVE), in percent: how "
                       "matrix-bound the work is while the GPU runs anything; wall-time utilisation is "
                       "gpu_mfma_util_percent.",
                       dev, d.mfma_busy));
    for (size_t x = 0; x < d.xcd_mfma_busy.size(); ++x) {
      out.push_back(xs("gpu_xcd_mfma_busy_active_percent", "MFMA busy share of active cycles per XCD, in percent.",
                       dev, d.xcd_mfma_busy[x]));
      out.back().labels.push_back({"xcd", std::to_string(x)});
    }
    for (const auto& [dt, tf] : d.mfma_tflops) {
      out.push_back(xs("gpu_mfma_tflops",
                       "Achieved MFMA throughput by operand type in TFLOP/s (512 x SQ_INSTS_VALU_MFMA_MOPS_<type> "
                       "over the counted interval; every process).",
                       dev, tf));
      out.back().labels.push_back({"dtype", dt});
    }
    if (!std::isnan(d.occupancy))
      out.push_back(xs("gpu_occupancy_percent", "Resident waves / max waves % from SQ_WAVE_CYCLES (only when configured; counts the profiling process own waves).", dev,
                       d.occupancy));
    if (!std::isnan(d.gui_active))
      out.push_back(xs("gpu_gui_active_percent",
                       "GRBM_GUI_ACTIVE / GRBM_COUNT in percent: a share of CYCLES (the clock drops while idle, so it "
                       "reads above the wall-time activity for bursty loads).",
                       dev, d.gui_active));
    out.push_back(xs("gpu_pmc_window_seconds", "Counted time behind the last PMC sample.", dev, d.span_s));
    if (!std::isnan(d.coverage))
      out.push_back(xs("gpu_pmc_coverage_ratio",
                       "Counted time / wall time between PMC samples (1 = continuous counting; window mode: "
                       "window / period).",
                       dev, std::min(1.0, d.coverage)));
  }
  out.push_back(xs("gpumon_pmc_up", "1 if the last PMC step produced values (0: counters unavailable, e.g. held by "
                                    "another profiler; the pmc series are withdrawn meanwhile).",
                   -1, pmc_up_ ? 1.0 : 0.0));
  out.push_back(xs("gpumon_pmc_errors_total", "Failed PMC samples.", -1, static_cast<double>(pmc_errors_.load()),
                   "counter"));
  out.push_back(xs("gpumon_pmc_resets_total",
                   "Continuous-counting intervals dropped because the counts went backwards (contexts restarted "
                   "underneath the exporter).",
                   -1, static_cast<double>(pmc_resets_.load()), "counter"));
  ex_->set_extra("pmc", std::move(out));
}

// Interruptible sleep to a monotonic deadline, in <= 20 ms system_clock slices: a steady_clock
// wait compiles to pthread_cond_clockwait, which the toolchain's TSan does not intercept (it then
// reports the waiting thread as still holding the mutex). Same idiom as Exporter::sample_devices.
void OnDevice::sleep_until(int64_t deadline_ns) {
  std::unique_lock<std::mutex> lk(wait_mu_);
  while (running_) {
    const int64_t left = deadline_ns - mono_ns();
    if (left <= 0) return;
    wait_cv_.wait_until(lk, std::chrono::system_clock::now() +
                                std::chrono::nanoseconds(std::min<int64_t>(left, 20'000'000)));
  }
}

void OnDevice::pmc_loop() {
  while (running_) {
    const int64_t t0 = mono_ns();
    pmc_step();
    sleep_until(t0 + static_cast<int64_t>(cfg_.pmc_every_s * 1e9));
  }
}

// ---------------------------------------------------------------------------------------------
// K1 probe

// One probe per exported device that the probe's runtime can see. Called at start and, while the
// exporter's backend has not come up yet (empty statics), again on later steps. Devices are paired
// with the runtime's HIP ordinals by PCI address where the plugin reports it: the exporter's
// hip_id is node-wide, the ordinals follow HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES of the
// process (gpumon/parallel/devmap.py does the same for the bench). Without it, by hip_id.
bool OnDevice::create_probes(std::string* err) {
  if (!probes_.empty()) return true;
  char ebuf[512] = {0};
  const int n_hip = probe_lib_->probe_count();
  std::map<std::string, int> ordinal_of;  // normalised BDF -> HIP ordinal
  if (probe_lib_->probe_pci)
    for (int o = 0; o < n_hip; ++o) {
      char b[64] = {0};
      if (probe_lib_->probe_pci(o, b, sizeof b) > 0) {
        const std::string nb = normalize_bdf(b);
        if (!nb.empty()) ordinal_of[nb] = o;
      }
    }
  probe_by_bdf_ = !ordinal_of.empty();
  std::vector<ProbeDev> made;
  for (const auto& s : ex_->statics()) {
    int ord = s.hip_id;
    if (probe_by_bdf_) {
      const auto it = ordinal_of.find(normalize_bdf(s.bdf));
      if (it == ordinal_of.end()) continue;  // a GPU the probe's runtime does not see
      ord = it->second;
    }
    if (ord < 0 || ord >= n_hip) continue;
    ProbeDev d;
    d.dev = s.index;
    d.handle = probe_lib_->probe_create(ord, cfg_.probe_blocks, 4, cfg_.probe_spin_ticks, ebuf, sizeof ebuf);
    if (!d.handle) {
      *err = std::string("probe create on hip device ") + std::to_string(ord) + ": " + ebuf;
      for (auto& p : made) probe_lib_->probe_destroy(static_cast<gpumon_probe*>(p.handle));
      return false;
    }
    made.push_back(std::move(d));
  }
  probes_ = std::move(made);
  return true;
}

void OnDevice::probe_step() {
  std::lock_guard<std::mutex> g(probe_mu_);
  probe_steps_++;
  if (helper_ && !pmc_lib_) export_helper();  // the PMC step refreshes it when both run
  if (!helper_check()) {
    for (auto& p : probes_) p.timeouts++, probe_timeouts_++;
    export_probe();
    return;
  }
  if (helper_ && helper_gen_.load() != probe_gen_seen_) {
    // a respawned helper: the old handles named probes in the dead process (nothing to free here)
    probes_.clear();
    probe_gen_seen_ = helper_gen_.load();
  }
  if (probes_.empty()) {
    std::string err;
    if (!create_probes(&err)) GPUMON_LOG(LogLevel::kWarn, "ondevice", err);
  }
  const int n = static_cast<int>(probes_.size());
  std::vector<int> got(n, 0);
  std::vector<gpumon_probe_result_t> res(n);
  bool failed = false;  // the helper did not answer: every probe's step is lost
  if (probe_lib_->probe_cycle) {
    std::vector<gpumon_probe*> hs(n);
    std::vector<int> pend(n);
    for (int k = 0; k < n; ++k) {
      hs[k] = static_cast<gpumon_probe*>(probes_[k].handle);
      pend[k] = probes_[k].pending;
    }
    if (probe_lib_->probe_cycle(hs.data(), n, cfg_.probe_timeout_s, pend.data(), got.data(), res.data()))
      for (int k = 0; k < n; ++k) probes_[k].pending = pend[k];
    else
      failed = true;
  } else {
    for (auto& p : probes_)
      if (p.pending < 0) p.pending = probe_lib_->probe_launch(static_cast<gpumon_probe*>(p.handle));
    const int64_t deadline = mono_ns() + static_cast<int64_t>(cfg_.probe_timeout_s * 1e9);
    for (int k = 0; k < n; ++k) {
      auto& p = probes_[k];
      if (p.pending < 0) continue;
      const double left = std::max(0.0, (deadline - mono_ns()) * 1e-9);
      got[k] = probe_lib_->probe_wait(static_cast<gpumon_probe*>(p.handle), p.pending, left, &res[k]) == 1;
      if (got[k]) p.pending = -1;
    }
  }
  for (int k = 0; k < n; ++k) {
    auto& p = probes_[k];
    const gpumon_probe_result_t& r = res[k];
    if (got[k]) {
      p.pending = -1;
      p.have = true;
      p.latency_s = r.host_latency_s;
      p.span_s = r.gpu_span_s;
      p.unique_cus = r.unique_cus;
      p.stale += static_cast<uint64_t>(std::max(0, r.stale_records));
      p.xcc_blocks.assign(r.xcc_blocks, r.xcc_blocks + GPUMON_PROBE_MAX_XCC);
      p.xcc_mhz.assign(r.xcc_clock_mhz, r.xcc_clock_mhz + GPUMON_PROBE_MAX_XCC);
      p.xcc_slot.assign(r.xcc_wave_slot, r.xcc_wave_slot + GPUMON_PROBE_MAX_XCC);
      p.slot_mean = r.wave_slot_mean;
      probe_done_++;
    } else if (p.pending >= 0 || failed) {
      p.timeouts++;
      probe_timeouts_++;
    }
  }
  export_probe();
}

constexpr const char* kSlotHelp =
    "Mean lowest wave slot a probe wave got per SIMD: wave slots held by other work at probe launch. Exact "
    "only for PERSISTENT partial loads; short kernels free their slots between launches and read far low (a "
    "saturating burn reads ~1 of 8). For occupancy use gpu_cu_occupancy_percent (KFD, interval mean).";

void OnDevice::export_probe() {
  std::vector<ExtraSeries> out;
  const std::vector<int> xcds = ex_->xcd_counts();
  for (const auto& p : probes_) {
    out.push_back(xs("gpu_probe_pending", "1 if the last probe launch has not completed yet.", p.dev,
                     p.pending >= 0 ? 1 : 0));
    out.push_back(xs("gpu_probe_timeouts_total", "Probe polls that timed out (GPU saturated or hung).", p.dev,
                     static_cast<double>(p.timeouts), "counter"));
    out.push_back(xs("gpu_probe_stale_records_total", "Probe records not visible when the arrival flag was.", p.dev,
                     static_cast<double>(p.stale), "counter"));
    if (!p.have) continue;
    out.push_back(xs("gpu_probe_latency_seconds", "Probe host launch -> all workgroups arrived (pinned ring).", p.dev,
                     p.latency_s));
    out.push_back(xs("gpu_probe_kernel_span_seconds", "Probe first start -> last end on the GPU 100 MHz clock.", p.dev,
                     p.span_s));
    out.push_back(xs("gpu_probe_unique_cus", "Distinct compute units that ran probe workgroups.", p.dev, p.unique_cus));
    out.push_back(xs("gpu_probe_wave_slot_mean", kSlotHelp, p.dev, p.slot_mean));
    // XCD liveness: every XCD the device has gets a gpu_probe_xcd_blocks sample, 0 when none of
    // the probe's workgroups ran there (an alertable value instead of a vanished series)
    const int n_xcd = p.dev < static_cast<int>(xcds.size()) ? xcds[p.dev] : 0;
    for (size_t x = 0; x < p.xcc_blocks.size(); ++x) {
      if (!p.xcc_blocks[x]) {
        if (static_cast<int>(x) < n_xcd) {
          out.push_back(xs("gpu_probe_xcd_blocks", "Probe workgroups executed per XCD (liveness: 0 = the XCD ran none of them).", p.dev, 0.0));
          out.back().labels.push_back({"xcd", std::to_string(x)});
        }
        continue;
      }
      out.push_back(xs("gpu_probe_xcd_blocks", "Probe workgroups executed per XCD (liveness: 0 = the XCD ran none of them).", p.dev, p.xcc_blocks[x]));
      out.back().labels.push_back({"xcd", std::to_string(x)});
      out.push_back(xs("gpu_probe_xcd_clock_mhz", "Effective shader clock per XCD measured in-kernel.", p.dev,
                       p.xcc_mhz[x]));
      out.back().labels.push_back({"xcd", std::to_string(x)});
      out.push_back(xs("gpu_probe_xcd_wave_slot_mean", kSlotHelp, p.dev, p.xcc_slot[x]));
      out.back().labels.push_back({"xcd", std::to_string(x)});
    }
  }
  ex_->set_extra("probe", std::move(out));
}

void OnDevice::probe_loop() {
  while (running_) {
    const int64_t t0 = mono_ns();
    probe_step();
    sleep_until(t0 + static_cast<int64_t>(cfg_.probe_every_s * 1e9));
  }
}

}  // namespace gpumon
