"""Device-wide PMC sampling (rocprofiler-sdk device counting) -> MFMA busy / occupancy series.

Exported per GPU (derived with the gfx9xx formulas ROCm 7.2 falls back to for gfx950, see
MI355X_MICROARCH.md §rocprofv3 PMC slots):

* ``gpu_mfma_busy_percent``      = 100 * sum(SQ_VALU_MFMA_BUSY_CYCLES) / (max(GRBM_GUI_ACTIVE) * SIMDs)
* ``gpu_xcd_mfma_busy_percent``  = the same per XCC (when the counter carries an XCC dimension)
* ``gpu_occupancy_percent``      = 400 * sum(SQ_WAVE_CYCLES) / max(GRBM_GUI_ACTIVE) / CUs / max_waves_per_cu
* ``gpu_gui_active_percent``     = 100 * max(GRBM_GUI_ACTIVE) / max(GRBM_COUNT)
* ``gpu_pmc_window_seconds``     — counting window per sample (duty cycle = window / interval)

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

DEFAULT_COUNTERS = ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]


def pmc_module():
    try:
        return importlib.import_module("gpumon._pmc")
    except ImportError as e:
        raise ImportError("gpumon._pmc is not built; run `make pmc`") from e


def derive(raw: Dict[str, dict], agent: dict) -> Dict[str, object]:
    """Turn reduced counter values into percentages (pure function, unit-tested on CPU)."""
    out: Dict[str, object] = {}
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
                res[dev] = derive(raw, self.agents[self.map[dev]])
                res[dev]["raw"] = raw
            self.last.update(res)
            self._export()
            return res
        for dev, ai in self.map.items():
            try:
                raw = self.P.sample(ai, self.counters, self.window_s)
                res[dev] = derive(raw, self.agents[ai])
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
                add("gpu_mfma_busy_percent", "MFMA pipe busy % (rocprofiler device counting).", dev, d["mfma_busy"])
            for x, v in enumerate(d.get("xcd_mfma_busy", [])):
                add("gpu_xcd_mfma_busy_percent", "MFMA pipe busy % per XCD.", dev, v, {"xcd": str(x)})
            if "occupancy" in d:
                add("gpu_occupancy_percent", "Resident waves / max waves % (rocprofiler device counting).", dev,
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
