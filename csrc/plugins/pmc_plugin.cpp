// libgpumon_pmc.so — device-wide hardware counters on MI355X via rocprofiler-sdk device counting.
//
// Why this exists: SQ/GRBM performance counters are privileged registers programmed through the
// driver / aqlprofile; shader code (the K1 probe kernel) cannot read them on CDNA4. The north star
// asks for MFMA-busy and occupancy percentages without host-side stalls: device counting samples
// the whole GPU (every queue, every process) from a host thread, with no kernel instrumentation and
// no synchronisation with the workload.
//
// Flow: rocprofiler_force_configure() registers this library as a tool BEFORE the HSA runtime
// initialises; tool_init() creates one context per GPU agent with the device counting service;
// hsa_init() then brings the runtime up. A sample = start contexts -> window -> read -> stop, so a
// value is the counter delta over `window_s` (duty cycle window/interval). Values are reduced per
// counter (sum / max over instances) and per XCC when the counter has an XCC dimension.
//
// C ABI in ondevice_abi.h; users: bin/gpumon-exporter and gpumon._core (csrc/core/ondevice.cpp,
// dlopen) and the gpumon._pmc Python module (csrc/pmc/pmc_module.cpp, linked).
#include <hsa/hsa.h>
#include <rocprofiler-sdk/internal_threading.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <dirent.h>

#include <algorithm>
#include <chrono>
#include <set>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ondevice_abi.h"

#define GPUMON_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct Agent {
  rocprofiler_agent_v0_t info{};
  rocprofiler_context_id_t ctx{};
  rocprofiler_counter_config_id_t active{};
  std::map<std::string, rocprofiler_counter_id_t> supported;
  std::map<std::vector<std::string>, std::pair<rocprofiler_counter_config_id_t, size_t>> profiles;
  std::map<uint64_t, std::string> id2name;
  std::map<uint64_t, rocprofiler_counter_dimension_id_t> xcc_dim;  // counter id -> XCC dim id
};

std::mutex g_mu;       // agent tables + counter configs
std::mutex g_sample;   // one counting window at a time (contexts are per agent, shared by callers)
std::vector<std::unique_ptr<Agent>> g_agents;
std::string g_err;
bool g_configured = false;
bool g_hsa = false;

// Continuous counting (gpumon_pmc_read_running): contexts left started between reads. Guarded by
// g_sample, like every start/stop/read.
struct Running {
  std::vector<int> agents;
  std::vector<std::string> counters;
  bool on = false;
};
Running g_run;

std::string st_str(rocprofiler_status_t s) { return rocprofiler_get_status_string(s); }

// Threads the runtimes create for us get names saying which step created them ("pmc-hsa-0",
// "pmc-ctx-1", ...): per-thread CPU of the exporter is then attributable (tools/thread_cpu.py).
std::set<int> task_ids() {
  std::set<int> s;
  if (DIR* d = opendir("/proc/self/task")) {
    while (dirent* e = readdir(d))
      if (e->d_name[0] >= '0' && e->d_name[0] <= '9') s.insert(atoi(e->d_name));
    closedir(d);
  }
  return s;
}

void name_new_threads(const std::set<int>& before, const char* step) {
  int k = 0;
  for (int t : task_ids()) {
    if (before.count(t)) continue;
    char path[64], name[16], cur[32] = {0};
    snprintf(path, sizeof path, "/proc/self/task/%d/comm", t);
    if (FILE* f = fopen(path, "r")) {  // already named (an inner step named it): keep
      const bool named = fgets(cur, sizeof cur, f) && strncmp(cur, "pmc-", 4) == 0;
      fclose(f);
      if (named) continue;
    }
    snprintf(name, sizeof name, "pmc-%s-%d", step, k++);
    if (FILE* f = fopen(path, "w")) {
      fputs(name, f);
      fclose(f);
    }
  }
}

void check(rocprofiler_status_t s, const char* what) {
  if (s != ROCPROFILER_STATUS_SUCCESS) throw std::runtime_error(std::string(what) + ": " + st_str(s));
}

void set_err(char* err, size_t n, const std::string& m) {
  if (err && n) snprintf(err, n, "%s", m.c_str());
}

// Threads rocprofiler-sdk creates internally for a runtime library are named "pmc-rp<lib>-N" (see
// name_new_threads): the creating library of every runtime thread in the exporter is then known.
std::set<int> g_rp_before;
const char* lib_tag(rocprofiler_runtime_library_t lib) {
  switch (lib) {
    case ROCPROFILER_LIBRARY: return "rprof";
    case ROCPROFILER_HSA_LIBRARY: return "rphsa";
    case ROCPROFILER_HIP_LIBRARY: return "rphip";
    default: return "rpoth";
  }
}

int tool_init(rocprofiler_client_finalize_t, void*) {
  try {
    std::vector<rocprofiler_agent_v0_t> agents;
    check(rocprofiler_query_available_agents(
              ROCPROFILER_AGENT_INFO_VERSION_0,
              [](rocprofiler_agent_version_t, const void** arr, size_t n, void* ud) {
                auto* v = static_cast<std::vector<rocprofiler_agent_v0_t>*>(ud);
                for (size_t i = 0; i < n; ++i) {
                  auto* a = static_cast<const rocprofiler_agent_v0_t*>(arr[i]);
                  if (a->type == ROCPROFILER_AGENT_TYPE_GPU) v->push_back(*a);
                }
                return ROCPROFILER_STATUS_SUCCESS;
              },
              sizeof(rocprofiler_agent_v0_t), &agents),
          "query_available_agents");
    const char* dbg = getenv("GPUMON_PMC_DEBUG_INIT");  // diagnosis of runtime threads (tools/thread_cpu.py)
    const bool no_ctx = dbg && strcmp(dbg, "no-contexts") == 0;
    const bool no_svc = dbg && strcmp(dbg, "no-service") == 0;
    for (const auto& a : agents) {
      if (no_ctx) break;
      auto A = std::make_unique<Agent>();
      A->info = a;
      check(rocprofiler_create_context(&A->ctx), "create_context");
      if (no_svc) {
        g_agents.push_back(std::move(A));
        continue;
      }
      check(rocprofiler_configure_device_counting_service(
                A->ctx, rocprofiler_buffer_id_t{0}, a.id,
                [](rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set,
                   void* ud) {
                  auto* ag = static_cast<Agent*>(ud);
                  if (ag->active.handle != 0) set(ctx, ag->active);
                },
                A.get()),
            "configure_device_counting_service");
      g_agents.push_back(std::move(A));
    }
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
  return 0;
}

void tool_fini(void*) {}

rocprofiler_tool_configure_result_t* configure(uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
  id->name = "gpumon-pmc";
  rocprofiler_at_internal_thread_create(
      [](rocprofiler_runtime_library_t, void*) { g_rp_before = task_ids(); },
      [](rocprofiler_runtime_library_t lib, void*) { name_new_threads(g_rp_before, lib_tag(lib)); },
      static_cast<int>(ROCPROFILER_LIBRARY | ROCPROFILER_HSA_LIBRARY | ROCPROFILER_HIP_LIBRARY |
                       ROCPROFILER_MARKER_LIBRARY | ROCPROFILER_RCCL_LIBRARY),
      nullptr);

  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                 &tool_fini, nullptr};
  return &cfg;
}

// caller holds g_mu
void load_supported(Agent& A) {
  if (!A.supported.empty()) return;
  std::vector<rocprofiler_counter_id_t> ids;
  check(rocprofiler_iterate_agent_supported_counters(
            A.info.id,
            [](rocprofiler_agent_id_t, rocprofiler_counter_id_t* c, size_t n, void* ud) {
              auto* v = static_cast<std::vector<rocprofiler_counter_id_t>*>(ud);
              v->insert(v->end(), c, c + n);
              return ROCPROFILER_STATUS_SUCCESS;
            },
            &ids),
        "iterate_agent_supported_counters");
  for (auto id : ids) {
    rocprofiler_counter_info_v1_t info{};
    info.size = sizeof(info);
    if (rocprofiler_query_counter_info(id, ROCPROFILER_COUNTER_INFO_VERSION_1, &info) != ROCPROFILER_STATUS_SUCCESS)
      continue;
    A.supported[info.name] = id;
    A.id2name[id.handle] = info.name;
    for (uint64_t d = 0; d < info.dimensions_count; ++d) {
      std::string dn = info.dimensions[d]->name;
      if (dn == "DIMENSION_XCC" || dn == "XCC") A.xcc_dim[id.handle] = info.dimensions[d]->id;  // 7.2: DIMENSION_XCC
    }
  }
}

Agent* agent_locked(int agent) {
  if (agent < 0 || agent >= static_cast<int>(g_agents.size())) throw std::out_of_range("pmc agent index");
  Agent* A = g_agents[agent].get();
  load_supported(*A);
  return A;
}

// Resolve (and cache) the counter config for `counters` on `agent`; returns the record count.
size_t prepare(int agent, const std::vector<std::string>& counters, Agent** out) {
  std::lock_guard<std::mutex> g(g_mu);
  Agent* A = agent_locked(agent);
  auto it = A->profiles.find(counters);
  if (it == A->profiles.end()) {
    std::vector<rocprofiler_counter_id_t> ids;
    size_t expect = 0;
    for (const auto& c : counters) {
      auto s = A->supported.find(c);
      if (s == A->supported.end()) throw std::invalid_argument("counter not supported: " + c);
      ids.push_back(s->second);
      rocprofiler_counter_info_v1_t info{};
      info.size = sizeof(info);
      check(rocprofiler_query_counter_info(s->second, ROCPROFILER_COUNTER_INFO_VERSION_1, &info),
            "query_counter_info");
      expect += info.dimensions_instances_count;
    }
    rocprofiler_counter_config_id_t cfg{};
    check(rocprofiler_create_counter_config(A->info.id, ids.data(), ids.size(), &cfg), "create_counter_config");
    it = A->profiles.emplace(counters, std::make_pair(cfg, expect)).first;
  }
  A->active = it->second.first;
  *out = A;
  return it->second.second;
}

// Per counter: sum / max / count over all dimension instances, plus per-XCC sums.
void reduce(const Agent& A, const std::vector<rocprofiler_counter_record_t>& recs,
            const std::vector<std::string>& counters, gpumon_pmc_value_t* out) {
  for (size_t c = 0; c < counters.size(); ++c) out[c] = gpumon_pmc_value_t{};
  for (const auto& r : recs) {
    rocprofiler_counter_id_t cid{};
    rocprofiler_query_record_counter_id(r.id, &cid);
    auto nm = A.id2name.find(cid.handle);
    if (nm == A.id2name.end()) continue;
    auto pos_it = std::find(counters.begin(), counters.end(), nm->second);
    if (pos_it == counters.end()) continue;
    gpumon_pmc_value_t& v = out[pos_it - counters.begin()];
    v.max = v.n ? std::max(v.max, r.counter_value) : r.counter_value;
    v.sum += r.counter_value;
    v.n++;
    v.ok = 1;
    auto xd = A.xcc_dim.find(cid.handle);
    if (xd != A.xcc_dim.end()) {
      size_t pos = 0;
      if (rocprofiler_query_record_dimension_position(r.id, xd->second, &pos) == ROCPROFILER_STATUS_SUCCESS &&
          pos < GPUMON_PMC_MAX_XCC) {
        v.by_xcc[pos] += r.counter_value;
        v.n_xcc = std::max<int32_t>(v.n_xcc, static_cast<int32_t>(pos) + 1);
      }
    }
  }
}

// caller holds g_sample
void stop_running_locked() {
  if (!g_run.on) return;
  for (int a : g_run.agents)
    if (a >= 0 && a < static_cast<int>(g_agents.size())) rocprofiler_stop_context(g_agents[a]->ctx);
  g_run = Running{};
}

size_t copy_out(const std::string& s, char* buf, size_t n) {
  if (buf && n) snprintf(buf, n, "%s", s.c_str());
  return s.size() + 1;
}

}  // namespace

GPUMON_EXPORT int gpumon_pmc_abi_version(void) { return GPUMON_ONDEVICE_ABI; }

GPUMON_EXPORT int gpumon_pmc_init(char* err, size_t errlen) {
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_configured) {
    const auto before = task_ids();
    rocprofiler_status_t s = rocprofiler_force_configure(&configure);
    name_new_threads(before, "cfg");
    if (s != ROCPROFILER_STATUS_SUCCESS) {
      set_err(err, errlen, "rocprofiler_force_configure: " + st_str(s) +
                               " (HSA already initialised in this process? init must run first)");
      return -1;
    }
    g_configured = true;
  }
  if (!g_err.empty()) {
    set_err(err, errlen, "pmc tool_init: " + g_err);
    return -1;
  }
  if (!g_hsa) {
    const auto before = task_ids();
    const hsa_status_t hs = hsa_init();
    name_new_threads(before, "hsa");
    if (hs != HSA_STATUS_SUCCESS) {
      set_err(err, errlen, "hsa_init failed");
      return -1;
    }
    g_hsa = true;
  }
  return static_cast<int>(g_agents.size());
}

GPUMON_EXPORT int gpumon_pmc_agent(int agent, gpumon_pmc_agent_t* out) {
  std::lock_guard<std::mutex> g(g_mu);
  if (agent < 0 || agent >= static_cast<int>(g_agents.size()) || !out) return -1;
  const auto& a = g_agents[agent]->info;
  *out = gpumon_pmc_agent_t{};
  out->node_id = a.node_id;
  out->logical_node_id = a.logical_node_id;
  out->drm_render_minor = a.drm_render_minor;
  out->cu_count = a.cu_count;
  out->simd_count = a.simd_count;
  out->num_xcc = a.num_xcc;
  out->max_waves_per_cu = a.max_waves_per_cu;
  snprintf(out->name, sizeof out->name, "%s", a.name ? a.name : "");
  snprintf(out->product_name, sizeof out->product_name, "%s", a.product_name ? a.product_name : "");
  return 0;
}

GPUMON_EXPORT size_t gpumon_pmc_supported(int agent, char* buf, size_t buflen) {
  std::lock_guard<std::mutex> g(g_mu);
  try {
    std::string s;
    for (const auto& kv : agent_locked(agent)->supported) s += kv.first + "\n";
    return copy_out(s, buf, buflen);
  } catch (const std::exception&) {
    return 0;
  }
}

GPUMON_EXPORT size_t gpumon_pmc_dimensions(int agent, const char* counter, char* buf, size_t buflen) {
  std::lock_guard<std::mutex> g(g_mu);
  try {
    Agent* A = agent_locked(agent);
    auto it = A->supported.find(counter ? counter : "");
    if (it == A->supported.end()) return 0;
    rocprofiler_counter_info_v1_t info{};
    info.size = sizeof(info);
    check(rocprofiler_query_counter_info(it->second, ROCPROFILER_COUNTER_INFO_VERSION_1, &info), "query_counter_info");
    std::string s;
    for (uint64_t d = 0; d < info.dimensions_count; ++d)
      s += std::string(info.dimensions[d]->name) + ":" + std::to_string(info.dimensions[d]->instance_size) + "\n";
    return copy_out(s, buf, buflen);
  } catch (const std::exception&) {
    return 0;
  }
}

// Every listed agent counts over the SAME window: on an 8-GPU node one PMC step costs one window
// instead of eight back-to-back ones.
GPUMON_EXPORT int gpumon_pmc_sample_many(const int* agents, int n_agents, const char* const* counters, int n_counters,
                                         double window_s, gpumon_pmc_value_t* out, int32_t* ok, char* err,
                                         size_t errlen) {
  if (n_agents <= 0 || n_counters <= 0 || !agents || !counters || !out || !ok) {
    set_err(err, errlen, "pmc sample: empty request");
    return -1;
  }
  std::vector<std::string> names(counters, counters + n_counters);
  std::lock_guard<std::mutex> sg(g_sample);
  stop_running_locked();  // a windowed sample owns the contexts: continuous counting ends here
  std::vector<Agent*> As(n_agents, nullptr);
  std::vector<std::vector<rocprofiler_counter_record_t>> recs(n_agents);
  try {
    for (int k = 0; k < n_agents; ++k) recs[k].resize(std::max<size_t>(prepare(agents[k], names, &As[k]), 1));
  } catch (const std::exception& e) {
    set_err(err, errlen, e.what());
    return -1;
  }
  int started = 0;
  const auto before = task_ids();
  for (; started < n_agents; ++started)
    if (rocprofiler_start_context(As[started]->ctx) != ROCPROFILER_STATUS_SUCCESS) break;
  name_new_threads(before, "ctx");
  if (started == n_agents) std::this_thread::sleep_for(std::chrono::duration<double>(window_s));
  for (int k = 0; k < n_agents; ++k) {
    ok[k] = 0;
    if (k >= started) continue;
    size_t cnt = recs[k].size();
    if (rocprofiler_sample_device_counting_service(As[k]->ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, recs[k].data(),
                                                   &cnt) != ROCPROFILER_STATUS_SUCCESS)
      continue;
    recs[k].resize(cnt);
    ok[k] = 1;
  }
  for (int k = 0; k < started; ++k) rocprofiler_stop_context(As[k]->ctx);
  for (int k = 0; k < n_agents; ++k) {
    if (ok[k]) reduce(*As[k], recs[k], names, out + static_cast<size_t>(k) * n_counters);
    else
      for (int c = 0; c < n_counters; ++c) out[static_cast<size_t>(k) * n_counters + c] = gpumon_pmc_value_t{};
  }
  return 0;
}

// Continuous counting: the first call starts the contexts of `agents` with `counters`; later calls
// with the same request read them WITHOUT stopping, so no interval goes uncounted between reads.
// A different request (agents or counters) restarts the contexts. Every read returns the service's
// raw values for the running context; the caller works out the interval values (the service's
// read semantics on MI355X are measured in profiles/r2_pmc_continuous.md). *started = 1 when this
// call (re)started the contexts (its values cover only the instant since the start).
GPUMON_EXPORT int gpumon_pmc_read_running(const int* agents, int n_agents, const char* const* counters,
                                          int n_counters, gpumon_pmc_value_t* out, int32_t* ok, int32_t* started,
                                          char* err, size_t errlen) {
  if (n_agents <= 0 || n_counters <= 0 || !agents || !counters || !out || !ok) {
    set_err(err, errlen, "pmc read: empty request");
    return -1;
  }
  std::vector<int> ag(agents, agents + n_agents);
  std::vector<std::string> names(counters, counters + n_counters);
  std::lock_guard<std::mutex> sg(g_sample);
  if (g_run.on && (g_run.agents != ag || g_run.counters != names)) stop_running_locked();
  std::vector<Agent*> As(n_agents, nullptr);
  std::vector<std::vector<rocprofiler_counter_record_t>> recs(n_agents);
  try {
    for (int k = 0; k < n_agents; ++k) recs[k].resize(std::max<size_t>(prepare(agents[k], names, &As[k]), 1));
  } catch (const std::exception& e) {
    set_err(err, errlen, e.what());
    return -1;
  }
  if (started) *started = 0;
  if (!g_run.on) {
    const auto before = task_ids();
    int k = 0;
    for (; k < n_agents; ++k)
      if (rocprofiler_start_context(As[k]->ctx) != ROCPROFILER_STATUS_SUCCESS) break;
    name_new_threads(before, "ctx");
    if (k < n_agents) {
      for (int j = 0; j < k; ++j) rocprofiler_stop_context(As[j]->ctx);
      set_err(err, errlen, "pmc read: start_context failed on agent " + std::to_string(agents[k]) +
                               " (another profiler holds the device counters?)");
      return -1;
    }
    g_run.agents = ag;
    g_run.counters = names;
    g_run.on = true;
    if (started) *started = 1;
  }
  for (int k = 0; k < n_agents; ++k) {
    ok[k] = 0;
    size_t cnt = recs[k].size();
    if (rocprofiler_sample_device_counting_service(As[k]->ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, recs[k].data(),
                                                   &cnt) == ROCPROFILER_STATUS_SUCCESS) {
      recs[k].resize(cnt);
      ok[k] = 1;
      reduce(*As[k], recs[k], names, out + static_cast<size_t>(k) * n_counters);
    } else {
      for (int c = 0; c < n_counters; ++c) out[static_cast<size_t>(k) * n_counters + c] = gpumon_pmc_value_t{};
    }
  }
  return 0;
}

GPUMON_EXPORT void gpumon_pmc_stop_running(void) {
  std::lock_guard<std::mutex> sg(g_sample);
  stop_running_locked();
}
