// gpumon._pmc — device-wide hardware counters on MI355X via rocprofiler-sdk device counting.
//
// Why this exists: SQ/GRBM performance counters are privileged registers programmed through the
// driver / aqlprofile; shader code (the K1 probe kernel) cannot read them on CDNA4. The north star
// asks for MFMA-busy and occupancy percentages without host-side stalls: device counting samples
// the whole GPU (every queue, every process) from a host thread, with no kernel instrumentation and
// no synchronisation with the workload.
//
// Flow: rocprofiler_force_configure() registers this module as a tool BEFORE the HSA runtime
// initialises; tool_init() creates one context per GPU agent with the device counting service;
// hsa_init() then brings the runtime up. sample() = start context -> window -> read -> stop, so a
// sample is the counter delta over `window_s` (duty cycle window/interval). Values are reduced per
// counter (sum / max over instances) and per XCC when the counter has an XCC dimension.
#include <hsa/hsa.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace {

struct Agent {
  rocprofiler_agent_v0_t info{};
  rocprofiler_context_id_t ctx{};
  rocprofiler_counter_config_id_t active{};
  std::map<std::string, rocprofiler_counter_id_t> supported;
  std::map<std::vector<std::string>, std::pair<rocprofiler_counter_config_id_t, size_t>> profiles;
  std::map<uint64_t, std::string> id2name;
  std::map<uint64_t, rocprofiler_counter_dimension_id_t> xcc_dim;  // counter id -> XCC dim id
  std::map<uint64_t, bool> has_xcc;
};

std::mutex g_mu;
std::vector<std::unique_ptr<Agent>> g_agents;
std::string g_err;
bool g_configured = false;
bool g_hsa = false;
rocprofiler_client_finalize_t g_fini = nullptr;
rocprofiler_client_id_t* g_client = nullptr;

std::string st_str(rocprofiler_status_t s) { return rocprofiler_get_status_string(s); }

void check(rocprofiler_status_t s, const char* what) {
  if (s != ROCPROFILER_STATUS_SUCCESS) throw std::runtime_error(std::string(what) + ": " + st_str(s));
}

int tool_init(rocprofiler_client_finalize_t fini, void*) {
  g_fini = fini;
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
    for (const auto& a : agents) {
      auto A = std::make_unique<Agent>();
      A->info = a;
      check(rocprofiler_create_context(&A->ctx), "create_context");
      Agent* raw = A.get();
      check(rocprofiler_configure_device_counting_service(
                A->ctx, rocprofiler_buffer_id_t{0}, a.id,
                [](rocprofiler_context_id_t ctx, rocprofiler_agent_id_t, rocprofiler_device_counting_agent_cb_t set,
                   void* ud) {
                  auto* ag = static_cast<Agent*>(ud);
                  if (ag->active.handle != 0) set(ctx, ag->active);
                },
                raw),
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
  g_client = id;
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init,
                                                 &tool_fini, nullptr};
  return &cfg;
}

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
    bool found = false;
    for (uint64_t d = 0; d < info.dimensions_count; ++d) {
      std::string dn = info.dimensions[d]->name;
      if (dn == "DIMENSION_XCC" || dn == "XCC") {  // ROCm 7.2 names it DIMENSION_XCC
        A.xcc_dim[id.handle] = info.dimensions[d]->id;
        found = true;
      }
    }
    A.has_xcc[id.handle] = found;
  }
}

}  // namespace

// Resolve (and cache) the counter config for `counters` on `agent`; returns the record count.
static size_t prepare(int agent, const std::vector<std::string>& counters, Agent** out) {
  std::lock_guard<std::mutex> g(g_mu);
  if (agent < 0 || agent >= static_cast<int>(g_agents.size())) throw std::out_of_range("agent");
  Agent* A = g_agents[agent].get();
  load_supported(*A);
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
static py::dict reduce(const Agent& A, const std::vector<rocprofiler_counter_record_t>& recs) {
  std::map<std::string, double> sum, mx;
  std::map<std::string, uint64_t> cnt;
  std::map<std::string, std::map<size_t, double>> by_xcc;
  for (const auto& r : recs) {
    rocprofiler_counter_id_t cid{};
    rocprofiler_query_record_counter_id(r.id, &cid);
    auto nm = A.id2name.find(cid.handle);
    std::string name = nm == A.id2name.end() ? "UNKNOWN" : nm->second;
    sum[name] += r.counter_value;
    mx[name] = cnt[name] ? std::max(mx[name], r.counter_value) : r.counter_value;
    cnt[name]++;
    auto xd = A.xcc_dim.find(cid.handle);
    if (xd != A.xcc_dim.end()) {
      size_t pos = 0;
      if (rocprofiler_query_record_dimension_position(r.id, xd->second, &pos) == ROCPROFILER_STATUS_SUCCESS)
        by_xcc[name][pos] += r.counter_value;
    }
  }
  py::dict out;
  for (const auto& kv : sum) {
    py::dict d;
    d["sum"] = kv.second;
    d["max"] = mx[kv.first];
    d["n"] = cnt[kv.first];
    std::vector<double> xs;
    for (const auto& [pos, v] : by_xcc[kv.first]) {
      if (xs.size() <= pos) xs.resize(pos + 1, 0.0);
      xs[pos] = v;
    }
    d["by_xcc"] = xs;
    out[py::str(kv.first)] = d;
  }
  return out;
}

PYBIND11_MODULE(_pmc, m) {
  m.doc() = "gpumon device-wide PMC sampling (rocprofiler-sdk device counting service)";

  m.def("init", []() {
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_configured) {
      rocprofiler_status_t s = rocprofiler_force_configure(&configure);
      if (s != ROCPROFILER_STATUS_SUCCESS)
        throw std::runtime_error("rocprofiler_force_configure: " + st_str(s) +
                                 " (HSA already initialised in this process? init() must run first)");
      g_configured = true;
    }
    if (!g_err.empty()) throw std::runtime_error("pmc tool_init: " + g_err);
    if (!g_hsa) {
      hsa_status_t h = hsa_init();
      if (h != HSA_STATUS_SUCCESS) throw std::runtime_error("hsa_init failed");
      g_hsa = true;
    }
    return static_cast<int>(g_agents.size());
  });

  m.def("agents", []() {
    std::lock_guard<std::mutex> g(g_mu);
    py::list l;
    for (auto& A : g_agents) {
      py::dict d;
      d["node_id"] = A->info.node_id;
      d["logical_node_id"] = A->info.logical_node_id;
      d["name"] = A->info.name ? A->info.name : "";
      d["product_name"] = A->info.product_name ? A->info.product_name : "";
      d["cu_count"] = A->info.cu_count;
      d["simd_count"] = A->info.simd_count;
      d["num_xcc"] = A->info.num_xcc;
      d["max_waves_per_cu"] = A->info.max_waves_per_cu;
      d["drm_render_minor"] = A->info.drm_render_minor;
      l.append(d);
    }
    return l;
  });

  m.def("supported_counters", [](int agent) {
    std::lock_guard<std::mutex> g(g_mu);
    if (agent < 0 || agent >= static_cast<int>(g_agents.size())) throw std::out_of_range("agent");
    load_supported(*g_agents[agent]);
    std::vector<std::string> v;
    for (auto& kv : g_agents[agent]->supported) v.push_back(kv.first);
    return v;
  });

  m.def("counter_dimensions", [](int agent, const std::string& counter) {
    std::lock_guard<std::mutex> g(g_mu);
    if (agent < 0 || agent >= static_cast<int>(g_agents.size())) throw std::out_of_range("agent");
    load_supported(*g_agents[agent]);
    auto it = g_agents[agent]->supported.find(counter);
    if (it == g_agents[agent]->supported.end()) throw std::invalid_argument("counter not supported: " + counter);
    rocprofiler_counter_info_v1_t info{};
    info.size = sizeof(info);
    check(rocprofiler_query_counter_info(it->second, ROCPROFILER_COUNTER_INFO_VERSION_1, &info), "query_counter_info");
    py::list l;
    for (uint64_t d = 0; d < info.dimensions_count; ++d)
      l.append(py::make_tuple(std::string(info.dimensions[d]->name), info.dimensions[d]->instance_size));
    return l;
  });

  m.def(
      "sample",
      [](int agent, std::vector<std::string> counters, double window_s) {
        Agent* A = nullptr;
        size_t n = prepare(agent, counters, &A);
        std::vector<rocprofiler_counter_record_t> recs(std::max<size_t>(n, 1));
        rocprofiler_status_t st;
        {
          py::gil_scoped_release nogil;
          check(rocprofiler_start_context(A->ctx), "start_context");
          std::this_thread::sleep_for(std::chrono::duration<double>(window_s));
          size_t cnt = recs.size();
          st = rocprofiler_sample_device_counting_service(A->ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE, recs.data(), &cnt);
          rocprofiler_stop_context(A->ctx);
          recs.resize(cnt);
        }
        check(st, "sample_device_counting_service");
        return reduce(*A, recs);
      },
      py::arg("agent"), py::arg("counters"), py::arg("window_s") = 0.1);

  // Every listed agent counts over the SAME window: on an 8-GPU node one PMC step costs one
  // window instead of eight back-to-back ones.
  m.def(
      "sample_many",
      [](std::vector<int> agents, std::vector<std::string> counters, double window_s) {
        std::vector<Agent*> As(agents.size(), nullptr);
        std::vector<std::vector<rocprofiler_counter_record_t>> recs(agents.size());
        for (size_t k = 0; k < agents.size(); ++k)
          recs[k].resize(std::max<size_t>(prepare(agents[k], counters, &As[k]), 1));
        std::vector<rocprofiler_status_t> st(agents.size(), ROCPROFILER_STATUS_SUCCESS);
        {
          py::gil_scoped_release nogil;
          size_t started = 0;
          for (; started < As.size(); ++started)
            if (rocprofiler_start_context(As[started]->ctx) != ROCPROFILER_STATUS_SUCCESS) break;
          if (started == As.size()) std::this_thread::sleep_for(std::chrono::duration<double>(window_s));
          for (size_t k = 0; k < As.size(); ++k) {
            if (k >= started) {
              st[k] = ROCPROFILER_STATUS_ERROR;
              continue;
            }
            size_t cnt = recs[k].size();
            st[k] = rocprofiler_sample_device_counting_service(As[k]->ctx, {}, ROCPROFILER_COUNTER_FLAG_NONE,
                                                               recs[k].data(), &cnt);
            recs[k].resize(cnt);
          }
          for (size_t k = 0; k < started; ++k) rocprofiler_stop_context(As[k]->ctx);
        }
        py::list out;
        for (size_t k = 0; k < As.size(); ++k) {
          if (st[k] != ROCPROFILER_STATUS_SUCCESS) {
            out.append(py::none());
            continue;
          }
          out.append(reduce(*As[k], recs[k]));
        }
        return out;
      },
      py::arg("agents"), py::arg("counters"), py::arg("window_s") = 0.1,
      "sample() for several agents over one shared window; None for an agent that failed");
}
