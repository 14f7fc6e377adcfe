"""Device-wide PMC sampling (rocprofiler-sdk device counting) -> MFMA busy / throughput series.

Exported per GPU (derived with the gfx9xx formulas ROCm 7.2 falls back to for gfx950, see
MI355X_MICROARCH.md §rocprofv3 PMC slots):

* ``gpu_mfma_busy_active_percent``     = 100 * sum(SQ_VALU_MFMA_BUSY_CYCLES) / (max(GRBM_GUI_ACTIVE) * SIMDs)
* ``gpu_xcd_mfma_busy_active_percent`` = the same per XCC (when the counter carries an XCC dimension)

This runner (windowed counting, no wall-time MFMA utilisation) is the TEST ORACLE for the
production path, the native samplers of csrc/core/ondevice.cpp (continuous counting,
``gpu_mfma_util_percent``); `gpumon serve` uses the native one unless ``--ondevice python``.
* ``gpu_mfma_tflops{dtype}``     = 512 * sum(SQ_INSTS_VALU_MFMA_MOPS_<DTYPE>) / window / 1e12
  (achieved matrix-core throughput per operand type: bf16, f16, f8, f6f4, f32, f64, i8)
* ``gpu_gui_active_percent``     = 100 * max(GRBM_GUI_ACTIVE) / max(GRBM_COUNT)
* ``gpu_pmc_window_seconds``     — counting window per sample (duty cycle = window / interval)
* ``gpu_occupancy_percent``      = 400 * sum(SQ_WAVE_CYCLES) / max(GRBM_GUI_ACTIVE) / CUs / max_waves_per_cu,
  only when SQ_WAVE_CYCLES is configured explicitly: on ROCm 7.2 device counting the per-wave SQ
  counters (SQ_WAVES, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_LEVEL_WAVES, SQ_INSTS_*) count only the
  waves of the profiling process, while the per-SIMD ones above (MFMA busy, MFMA MOPS) count every
  process (measured on MI355X: profiles/r1_pmc_cross_process.md). An exporter never owns the
  workload, so the default set has no wave counters; occupancy comes from KFD instead
  (``gpu_cu_occupancy_percent``, ``pod_gpu_proc_cu_occupancy_percent``) and from the K1 probe.

``init()`` of the native module must run before anything initialises HSA/HIP in the process
(rocprofiler_force_configure); :class:`gpumon.monitor.GpuMonitor` starts the PMC runner first.
"""

from __future__ import annotations

import importlib
import logging
import threading
import time
from typing import Dict, List

log = logging.getLogger("gpumon.pmc")
TFLOPS_HELP = ("Achieved MFMA throughput by operand type in TFLOP/s (512 x SQ_INSTS_VALU_MFMA_MOPS_<type> over the "
               "counting window; every process).")

# 8 SQ + 2 GRBM: exactly one counting pass on gfx950 (8 SQ / 2 GRBM counter slots)
MFMA_DTYPES = ["BF16", "F16", "F8", "F6F4", "F32", "F64", "I8"]
DEFAULT_COUNTERS = (["SQ_VALU_MFMA_BUSY_CYCLES"] + ["SQ_INSTS_VALU_MFMA_MOPS_" + d for d in MFMA_DTYPES]
                    + ["GRBM_GUI_ACTIVE", "GRBM_COUNT"])
MOPS_FLOP = 512.0  # FLOP per SQ_INSTS_VALU_MFMA_MOPS_* unit


def pmc_module():
    try:
        return importlib.import_module("gpumon._pmc")
    except ImportError as e:
        raise ImportError("gpumon._pmc is not built; run `make pmc`") from e


def derive(raw: Dict[str, dict], agent: dict, window_s: float = 0.0) -> Dict[str, object]:
    """Turn reduced counter values into percentages / TFLOP/s (pure function, unit-tested on CPU;
    C++ twin: gpumon._core.pmc_derive)."""
    out: Dict[str, object] = {}
    if window_s > 0:
        tf = {k[len("SQ_INSTS_VALU_MFMA_MOPS_"):].lower(): MOPS_FLOP * v["sum"] / window_s / 1e12
              for k, v in raw.items() if k.startswith("SQ_INSTS_VALU_MFMA_MOPS_")}
        if tf:
            out["mfma_tflops"] = tf
    gui = raw.get("GRBM_GUI_ACTIVE", {}).get("max", 0.0)
    simds = agent.get("simd_count") or (agent.get("cu_count", 0) * 4)
    cus = agent.get("cu_count") or 0
    waves = agent.get("max_waves_per_cu") or 32
    if gui > 0 and "SQ_VALU_MFMA_BUSY_CYCLES" in raw and simds:
        m = raw["SQ_VALU_MFMA_BUSY_CYCLES"]
        out["mfma_busy"] = min(100.0, 100.0 * m["sum"] / (gui * simds))
        xs = m.get("by_xcc") or []
        if xs and len(xs) > 1:
            per = simds / len(xs)
            out["xcd_mfma_busy"] = [min(100.0, 100.0 * v / (gui * per)) for v in xs]
    if gui > 0 and "SQ_WAVE_CYCLES" in raw and cus:
        out["occupancy"] = min(100.0, 400.0 * raw["SQ_WAVE_CYCLES"]["sum"] / gui / cus / waves)
    cnt = raw.get("GRBM_COUNT", {}).get("max", 0.0)
    if cnt > 0:
        out["gui_active"] = min(100.0, 100.0 * gui / cnt)
    return out


class PmcRunner:
    def __init__(self, exporter, counters: List[str] = None, every_s: float = 1.0, window_s: float = 0.1):
        self.ex = exporter
        self.counters = list(counters or DEFAULT_COUNTERS)
        self.every_s = every_s
        self.window_s = min(window_s, every_s * 0.5)
        self.P = pmc_module()
        self.P.init()
        self.agents = self.P.agents()
        self.map: Dict[int, int] = {}   # exporter device index -> pmc agent index
        statics = exporter.statics()
        for s in statics:
            for ai, a in enumerate(self.agents):
                if s.get("drm_render") == a["drm_render_minor"] or (
                        s.get("drm_render", -1) < 0 and ai == s["index"]):
                    self.map[s["index"]] = ai
        self.errors = 0
        self.last: Dict[int, dict] = {}
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._th = None

    def step(self) -> Dict[int, dict]:
        # one counting context per agent may run at a time: serialise explicit + background calls
        with self._lock:
            return self._step()

    def _step(self) -> Dict[int, dict]:
        res = {}
        if len(self.map) > 1 and hasattr(self.P, "sample_many"):
            # all GPUs count over one shared window (8 GPUs: one 0.1 s window, not eight)
            devs = list(self.map)
            try:
                raws = self.P.sample_many([self.map[d] for d in devs], self.counters, self.window_s)
            except Exception as e:  # noqa: BLE001
                raws = [None] * len(devs)
                log.warning("pmc sample_many failed: %s", e)
            for dev, raw in zip(devs, raws):
                if raw is None:
                    self.errors += 1
                    continue
                res[dev] = derive(raw, self.agents[self.map[dev]], self.window_s)
                res[dev]["raw"] = raw
            self.last.update(res)
            self._export()
            return res
        for dev, ai in self.map.items():
            try:
                raw = self.P.sample(ai, self.counters, self.window_s)
                res[dev] = derive(raw, self.agents[ai], self.window_s)
                res[dev]["raw"] = raw
            except Exception as e:  # noqa: BLE001
                self.errors += 1
                log.warning("pmc sample failed on device %d: %s", dev, e)
        self.last.update(res)
        self._export()
        return res

    def _export(self):
        series = []

        def add(name, help_, dev, v, labels=None):
            series.append({"name": name, "help": help_, "dev": dev, "value": float(v), "labels": labels or {}})

        for dev, d in self.last.items():
            if "mfma_busy" in d:
                add("gpu_mfma_busy_active_percent", "MFMA busy share of active cycles (windowed, Python oracle).",
                    dev, d["mfma_busy"])
            for x, v in enumerate(d.get("xcd_mfma_busy", [])):
                add("gpu_xcd_mfma_busy_active_percent", "MFMA busy share of active cycles per XCD.", dev, v,
                    {"xcd": str(x)})
            for dt, v in sorted(d.get("mfma_tflops", {}).items()):
                add("gpu_mfma_tflops", TFLOPS_HELP, dev, v, {"dtype": dt})
            if "occupancy" in d:
                add("gpu_occupancy_percent", "Resident waves / max waves % from SQ_WAVE_CYCLES (only when configured; counts the profiling process own waves).", dev,
                    d["occupancy"])
            if "gui_active" in d:
                add("gpu_gui_active_percent", "GRBM GUI active % of the counting window.", dev, d["gui_active"])
            add("gpu_pmc_window_seconds", "PMC counting window per sample.", dev, self.window_s)
        series.append({"name": "gpumon_pmc_errors_total", "help": "Failed PMC samples.", "dev": -1,
                       "value": float(self.errors), "type": "counter", "labels": {}})
        self.ex.set_extra("pmc", series)

    def start(self):
        self._th = threading.Thread(target=self._loop, name="gpumon-pmc", daemon=True)
        self._th.start()
        return self

    def _loop(self):
        while not self._stop.is_set():
            t0 = time.monotonic()
            self.step()
            self._stop.wait(max(0.0, self.every_s - (time.monotonic() - t0)))

    def stop(self):
        self._stop.set()
        if self._th:
            self._th.join(timeout=5)
        self.ex.set_extra("pmc", [])
