// gpumon._pmc — Python view of lib/libgpumon_pmc.so (rocprofiler-sdk device counting on MI355X).
//
// The counting code lives in csrc/plugins/pmc_plugin.cpp behind the C ABI of ondevice_abi.h; this
// module links that library (rpath $ORIGIN/../lib), so a process that uses both this module and the
// native sampler in gpumon._core (which dlopen()s the same path) shares ONE tool registration.
// Used by the calibration tools (tools/pmc_check.py, tools/duty_calibration.py) and the GPU tests.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../plugins/ondevice_abi.h"

namespace py = pybind11;

namespace {

std::vector<std::string> split_lines(const std::string& s) {
  std::vector<std::string> v;
  std::istringstream is(s);
  for (std::string l; std::getline(is, l);)
    if (!l.empty()) v.push_back(l);
  return v;
}

py::dict to_dict(const std::vector<std::string>& names, const gpumon_pmc_value_t* vals) {
  py::dict out;
  for (size_t c = 0; c < names.size(); ++c) {
    const auto& v = vals[c];
    if (!v.ok) continue;
    py::dict d;
    d["sum"] = v.sum;
    d["max"] = v.max;
    d["n"] = v.n;
    d["by_xcc"] = std::vector<double>(v.by_xcc, v.by_xcc + v.n_xcc);
    out[py::str(names[c])] = d;
  }
  return out;
}

py::list sample_many(const std::vector<int>& agents, const std::vector<std::string>& counters, double window_s) {
  std::vector<const char*> cn;
  for (const auto& c : counters) cn.push_back(c.c_str());
  std::vector<gpumon_pmc_value_t> vals(agents.size() * counters.size());
  std::vector<int32_t> ok(agents.size(), 0);
  char err[512] = {0};
  int rc;
  {
    py::gil_scoped_release nogil;
    rc = gpumon_pmc_sample_many(agents.data(), static_cast<int>(agents.size()), cn.data(),
                                static_cast<int>(cn.size()), window_s, vals.data(), ok.data(), err, sizeof err);
  }
  if (rc != 0) {
    std::string m = err;
    if (m.find("not supported") != std::string::npos) throw py::value_error(m);
    if (m.find("agent index") != std::string::npos) throw py::index_error(m);
    throw std::runtime_error(m);
  }
  py::list out;
  for (size_t k = 0; k < agents.size(); ++k) {
    if (!ok[k]) out.append(py::none());
    else out.append(to_dict(counters, vals.data() + k * counters.size()));
  }
  return out;
}

py::dict read_running(const std::vector<int>& agents, const std::vector<std::string>& counters) {
  std::vector<const char*> cn;
  for (const auto& c : counters) cn.push_back(c.c_str());
  std::vector<gpumon_pmc_value_t> vals(agents.size() * counters.size());
  std::vector<int32_t> ok(agents.size(), 0);
  int32_t started = 0;
  char err[512] = {0};
  int rc;
  {
    py::gil_scoped_release nogil;
    rc = gpumon_pmc_read_running(agents.data(), static_cast<int>(agents.size()), cn.data(),
                                 static_cast<int>(cn.size()), vals.data(), ok.data(), &started, err, sizeof err);
  }
  if (rc != 0) throw std::runtime_error(err);
  py::list per;
  for (size_t k = 0; k < agents.size(); ++k) {
    if (!ok[k]) per.append(py::none());
    else per.append(to_dict(counters, vals.data() + k * counters.size()));
  }
  py::dict d;
  d["started"] = started != 0;
  d["agents"] = per;
  return d;
}

}  // namespace

PYBIND11_MODULE(_pmc, m) {
  m.doc() = "gpumon device-wide PMC sampling (rocprofiler-sdk device counting, lib/libgpumon_pmc.so)";

  m.def("init", []() {
    char err[512] = {0};
    int n = gpumon_pmc_init(err, sizeof err);
    if (n < 0) throw std::runtime_error(err);
    return n;
  });

  m.def("agents", []() {
    py::list l;
    gpumon_pmc_agent_t a;
    for (int i = 0; gpumon_pmc_agent(i, &a) == 0; ++i) {
      py::dict d;
      d["node_id"] = a.node_id;
      d["logical_node_id"] = a.logical_node_id;
      d["name"] = std::string(a.name);
      d["product_name"] = std::string(a.product_name);
      d["cu_count"] = a.cu_count;
      d["simd_count"] = a.simd_count;
      d["num_xcc"] = a.num_xcc;
      d["max_waves_per_cu"] = a.max_waves_per_cu;
      d["drm_render_minor"] = a.drm_render_minor;
      l.append(d);
    }
    return l;
  });

  m.def("supported_counters", [](int agent) {
    size_t n = gpumon_pmc_supported(agent, nullptr, 0);
    if (n == 0) throw py::index_error("agent");
    std::string buf(n, '\0');
    gpumon_pmc_supported(agent, &buf[0], n);
    return split_lines(buf.c_str());
  });

  m.def("counter_dimensions", [](int agent, const std::string& counter) {
    size_t n = gpumon_pmc_dimensions(agent, counter.c_str(), nullptr, 0);
    if (n == 0) throw py::value_error("counter not supported: " + counter);
    std::string buf(n, '\0');
    gpumon_pmc_dimensions(agent, counter.c_str(), &buf[0], n);
    py::list l;
    for (const auto& line : split_lines(buf.c_str())) {
      auto c = line.rfind(':');
      l.append(py::make_tuple(line.substr(0, c), std::stoull(line.substr(c + 1))));
    }
    return l;
  });

  m.def(
      "sample",
      [](int agent, std::vector<std::string> counters, double window_s) {
        py::list l = sample_many({agent}, counters, window_s);
        if (l[0].is_none()) throw std::runtime_error("sample_device_counting_service failed");
        return py::dict(l[0]);
      },
      py::arg("agent"), py::arg("counters"), py::arg("window_s") = 0.1);

  m.def("read_running", &read_running, py::arg("agents"), py::arg("counters"),
        "continuous counting: read running contexts without stopping them ({'started', 'agents'})");
  m.def("stop_running", []() {
    py::gil_scoped_release nogil;
    gpumon_pmc_stop_running();
  });
  m.def("sample_many", &sample_many, py::arg("agents"), py::arg("counters"), py::arg("window_s") = 0.1,
        "sample() for several agents over one shared window; None for an agent that failed");
}
