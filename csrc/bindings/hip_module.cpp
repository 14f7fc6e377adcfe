// pybind11 bindings: gpumon._hip (gfx950 kernels: K1 probe, K2 synthetic load).
// Pointers/streams are passed as integers (torch tensor .data_ptr(), torch.cuda stream handle) so
// the kernels can be checked against PyTorch fp32 references on the same tensors.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../hip/hip_api.h"

namespace py = pybind11;
using namespace gpumon_hip;

static void* P(uintptr_t x) { return reinterpret_cast<void*>(x); }

PYBIND11_MODULE(_hip, m) {
  m.doc() = "gpumon gfx950 HIP kernels (probe ring buffer + synthetic MFMA/HBM load)";
  m.def("device_count", &device_count);
  m.def("device_arch", &device_arch);
  m.def("device_cu_count", &device_cu_count);
  m.def("device_pci_bus_id", &device_pci_bus_id);

  m.def("mfma_tile", [](int dev, uintptr_t a, uintptr_t b, uintptr_t c, int iters, uintptr_t stream) {
    launch_mfma_tile(dev, P(a), P(b), static_cast<float*>(P(c)), iters, P(stream));
  }, py::arg("dev"), py::arg("a"), py::arg("b"), py::arg("c"), py::arg("iters"), py::arg("stream") = 0);
  m.def("mfma_burn", [](int dev, uintptr_t a, uintptr_t b, uintptr_t out, int blocks, int iters, uintptr_t stream,
                        int shape) {
    launch_mfma_burn(dev, P(a), P(b), static_cast<float*>(P(out)), blocks, iters, P(stream), shape);
  }, py::arg("dev"), py::arg("a"), py::arg("b"), py::arg("out"), py::arg("blocks"), py::arg("iters"),
     py::arg("stream") = 0, py::arg("shape") = 32);
  m.def("mfma_burn_dtype", [](int dev, const std::string& dtype, uintptr_t out, int blocks, int iters,
                              uintptr_t stream) {
    return launch_mfma_burn_dtype(dev, dtype, static_cast<float*>(P(out)), blocks, iters, P(stream));
  }, py::arg("dev"), py::arg("dtype"), py::arg("out"), py::arg("blocks"), py::arg("iters"), py::arg("stream") = 0,
     "MFMA burn of one matrix path (f16|fp8|f32|f64|i8|mxfp8|mxfp4); returns FLOP per launch");
  m.def("stream_copy", [](int dev, uintptr_t src, uintptr_t dst, size_t n16, int blocks, uintptr_t stream,
                          int unroll, int policy, bool span) {
    launch_stream_copy(dev, P(src), P(dst), n16, blocks, P(stream), unroll, policy, span);
  }, py::arg("dev"), py::arg("src"), py::arg("dst"), py::arg("n16"), py::arg("blocks") = 4096,
     py::arg("stream") = 0, py::arg("unroll") = 4, py::arg("policy") = 0, py::arg("span") = false);
  m.def("stream_triad", [](int dev, uintptr_t a, uintptr_t b, uintptr_t c, float s, size_t n, int blocks,
                           uintptr_t stream) {
    launch_stream_triad(dev, static_cast<const float*>(P(a)), static_cast<const float*>(P(b)),
                        static_cast<float*>(P(c)), s, n, blocks, P(stream));
  }, py::arg("dev"), py::arg("a"), py::arg("b"), py::arg("c"), py::arg("s"), py::arg("n"),
     py::arg("blocks") = 4096, py::arg("stream") = 0);

  py::class_<LoadGen>(m, "LoadGen")
      .def(py::init([](int dev, std::string kind, double duty, size_t hbm_bytes, int mfma_iters, int shape,
                       std::string dtype, double period_s) {
             auto g = std::make_unique<LoadGen>(dev, std::move(kind), duty, hbm_bytes, mfma_iters);
             g->set_mfma_shape(shape);
             g->set_mfma_dtype(std::move(dtype));
             g->set_period(period_s);
             return g;
           }),
           py::arg("dev"), py::arg("kind") = "mixed", py::arg("duty") = 1.0, py::arg("hbm_bytes") = size_t(1) << 30,
           py::arg("mfma_iters") = 8192, py::arg("mfma_shape") = 32, py::arg("mfma_dtype") = "bf16",
           py::arg("period_s") = 0.0)
      .def("start", [](LoadGen& g) {
        py::gil_scoped_release nogil;
        g.start();
      })
      .def("stop", [](LoadGen& g) {
        py::gil_scoped_release nogil;
        g.stop();
      })
      .def_property_readonly("running", &LoadGen::running)
      .def("stats", [](LoadGen& g) {
        LoadStats s = g.stats();
        py::dict d;
        d["launches"] = s.launches;
        d["busy_s"] = s.busy_s;
        d["flops"] = s.flops;
        d["bytes"] = s.bytes;
        d["mfma_s"] = s.mfma_s;
        d["hbm_s"] = s.hbm_s;
        d["wall_s"] = s.wall_s;
        d["tflops"] = s.mfma_s > 0 ? s.flops / s.mfma_s / 1e12 : 0.0;  // rate while MFMA batches ran
        d["tbps"] = s.hbm_s > 0 ? s.bytes / s.hbm_s / 1e12 : 0.0;      // rate while HBM batches ran
        d["tflops_wall"] = s.wall_s > 0 ? s.flops / s.wall_s / 1e12 : 0.0;  // averaged over wall time
        d["tbps_wall"] = s.wall_s > 0 ? s.bytes / s.wall_s / 1e12 : 0.0;
        return d;
      });

  py::class_<XgmiLoad>(m, "XgmiLoad")
      .def(py::init<int, int, size_t, std::string, int>(), py::arg("src"), py::arg("dst"),
           py::arg("nbytes") = size_t(256) << 20, py::arg("method") = "kernel", py::arg("blocks") = 512)
      .def("start", [](XgmiLoad& g) {
        py::gil_scoped_release nogil;
        g.start();
      })
      .def("stop", [](XgmiLoad& g) {
        py::gil_scoped_release nogil;
        g.stop();
      })
      .def_property_readonly("running", &XgmiLoad::running)
      .def("stats", [](XgmiLoad& g) {
        XgmiStats s = g.stats();
        py::dict d;
        d["copies"] = s.copies;
        d["bytes"] = s.bytes;
        d["busy_s"] = s.busy_s;
        d["wall_s"] = s.wall_s;
        d["GBps"] = s.busy_s > 0 ? s.bytes / s.busy_s / 1e9 : 0.0;       // while copying
        d["GBps_wall"] = s.wall_s > 0 ? s.bytes / s.wall_s / 1e9 : 0.0;  // averaged over wall time
        return d;
      });

  py::class_<PcieLoad>(m, "PcieLoad")
      .def(py::init<int, size_t, std::string, double>(), py::arg("dev"), py::arg("nbytes") = size_t(256) << 20,
           py::arg("direction") = "both", py::arg("duty") = 1.0)
      .def("start", [](PcieLoad& g) {
        py::gil_scoped_release nogil;
        g.start();
      })
      .def("stop", [](PcieLoad& g) {
        py::gil_scoped_release nogil;
        g.stop();
      })
      .def_property_readonly("running", &PcieLoad::running)
      .def("stats", [](PcieLoad& g) {
        PcieStats s = g.stats();
        py::dict d;
        d["copies"] = s.copies;
        d["h2d_bytes"] = s.h2d_bytes;
        d["d2h_bytes"] = s.d2h_bytes;
        d["bytes"] = s.h2d_bytes + s.d2h_bytes;
        d["busy_s"] = s.busy_s;
        d["wall_s"] = s.wall_s;
        d["GBps_wall"] = s.wall_s > 0 ? (s.h2d_bytes + s.d2h_bytes) / s.wall_s / 1e9 : 0.0;  // both directions
        return d;
      });

  py::class_<Probe>(m, "Probe")
      .def(py::init<int, int, int, int>(), py::arg("dev"), py::arg("blocks") = 1024, py::arg("slots") = 4,
           py::arg("spin_ticks") = 200)
      .def("launch", &Probe::launch)
      .def_property_readonly("blocks", &Probe::blocks)
      .def("poll", [](Probe& p, int slot, double timeout_s) -> py::object {
        ProbeResult r;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = timeout_s > 0 ? p.wait(slot, timeout_s, &r) : p.poll(slot, &r);
        }
        if (!ok) return py::none();
        py::dict d;
        d["seq"] = r.seq;
        d["blocks"] = r.blocks;
        d["arrived"] = r.arrived;
        d["host_latency_s"] = (r.host_done_ns - r.host_launch_ns) * 1e-9;
        d["gpu_span_s"] = r.gpu_span_ticks * 1e-8;
        d["xcc_blocks"] = r.xcc_blocks;
        d["xcc_clock_mhz"] = r.xcc_clock_mhz;
        d["unique_cus"] = r.unique_cus;
        d["xcc_wave_slot"] = r.xcc_wave_slot;
        d["wave_slot_mean"] = r.wave_slot_mean;
        d["stale_records"] = r.stale_records;
        py::list recs;
        for (const auto& x : r.records)
          recs.append(py::make_tuple(x.xcc_id, x.hw_id, x.t0_real, x.t1_real, x.c0, x.c1, x.seq, x.block));
        d["records"] = recs;
        return d;
      }, py::arg("slot"), py::arg("timeout_s") = 0.0);
}
