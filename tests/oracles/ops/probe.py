"""K1 probe runner: launches the gfx950 probe microkernel on every monitored GPU and exports its
pinned-ring-buffer results as ``gpu_probe_*`` series.

This Python runner is the TEST ORACLE of the production path, the native sampler in
csrc/core/ondevice.cpp (same plugin, same series); `gpumon serve` uses the native one unless
``--ondevice python``.

Per tick and device: one launch of ``blocks`` one-wave workgroups on a private non-blocking stream;
completion is detected by polling a host-pinned arrival word that the last wave writes once, after a
device-memory (L2) arrival counter reaches ``blocks`` (no hipDeviceSynchronize, no stall of the
workload; see csrc/hip/kernels.hip K1). Exported:

* ``gpu_probe_xcd_blocks{xcd}``       — workgroups that ran on each XCD (per-XCD liveness)
* ``gpu_probe_xcd_clock_mhz{xcd}``    — effective shader clock per XCD (Δs_memtime / Δs_memrealtime)
* ``gpu_probe_latency_seconds``       — host launch -> all workgroups arrived (queueing behind the
                                        workload is the contention signal)
* ``gpu_probe_kernel_span_seconds``   — first start -> last end on the GPU's 100 MHz clock
* ``gpu_probe_unique_cus``            — distinct (XCD, SE, CU) ids seen
* ``gpu_probe_wave_slot_mean`` / ``gpu_probe_xcd_wave_slot_mean{xcd}`` — per SIMD, the lowest
  HW_ID.WAVE_ID a probe wave was given, averaged: the SPI allocates the lowest free slot, so this is
  the number of wave slots other work held at launch (in-kernel resident-wave pressure; 0 idle)
* ``gpu_probe_pending`` / ``gpu_probe_timeouts_total`` / ``gpu_probe_stale_records_total``

SQ/GRBM perf counters are not readable from shader code on CDNA4; MFMA-busy and occupancy come
from :mod:`gpumon.ops.pmc` (rocprofiler-sdk device counting).
"""

from __future__ import annotations

import logging
import threading
import time
from typing import Dict, List

from gpumon._native import hip

log = logging.getLogger("gpumon.probe")
SLOT_HELP = "Mean lowest wave slot a probe wave got per SIMD (wave slots held by other work at probe launch)."


class ProbeRunner:
    def __init__(self, exporter, every_s: float = 1.0, blocks: int = 1024, spin_ticks: int = 200,
                 timeout_s: float = 0.5):
        self.ex = exporter
        self.every_s = every_s
        self.timeout_s = min(timeout_s, every_s)
        self._hip = hip()
        self.devs: List[dict] = [s for s in exporter.statics()]
        n_hip = self._hip.device_count()
        self.probes: Dict[int, object] = {}
        for s in self.devs:
            hid = s["hip_id"]
            if 0 <= hid < n_hip:
                self.probes[s["index"]] = self._hip.Probe(hid, blocks, 4, spin_ticks)
        self.pending: Dict[int, int] = {}
        self.timeouts: Dict[int, int] = {i: 0 for i in self.probes}
        self.stale: Dict[int, int] = {i: 0 for i in self.probes}
        self.last: Dict[int, dict] = {}
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._th = None

    def step(self) -> Dict[int, dict]:
        """Launch (if the previous launch completed) and collect one round; returns results.
        Serialised: the background thread and an explicit caller (``gpumon once``) may both call it."""
        with self._lock:
            return self._step()

    def _step(self) -> Dict[int, dict]:
        for i, p in self.probes.items():
            if i not in self.pending:
                slot = p.launch()
                if slot >= 0:
                    self.pending[i] = slot
        deadline = time.monotonic() + self.timeout_s
        out = {}
        for i, p in self.probes.items():
            if i not in self.pending:
                continue
            r = p.poll(self.pending[i], max(0.0, deadline - time.monotonic()))
            if r is not None:
                out[i] = r
                self.last[i] = r
                self.stale[i] += r.get("stale_records", 0)
                del self.pending[i]
            else:
                self.timeouts[i] += 1
        self._export()
        return out

    def _export(self):
        series = []

        def add(name, help_, dev, value, labels=None, typ="gauge"):
            series.append({"name": name, "help": help_, "dev": dev, "value": float(value), "labels": labels or {},
                           "type": typ})

        for i in self.probes:
            add("gpu_probe_pending", "1 if the last probe launch has not completed yet.", i, 1 if i in self.pending else 0)
            add("gpu_probe_timeouts_total", "Probe polls that timed out (GPU saturated or hung).", i,
                self.timeouts[i], typ="counter")
            add("gpu_probe_stale_records_total", "Probe records not visible when the arrival flag was.", i,
                self.stale[i], typ="counter")
            r = self.last.get(i)
            if not r:
                continue
            add("gpu_probe_latency_seconds", "Probe host launch -> all workgroups arrived (pinned ring).", i,
                r["host_latency_s"])
            add("gpu_probe_kernel_span_seconds", "Probe first start -> last end on the GPU 100 MHz clock.", i,
                r["gpu_span_s"])
            add("gpu_probe_unique_cus", "Distinct compute units that ran probe workgroups.", i, r["unique_cus"])
            add("gpu_probe_wave_slot_mean", SLOT_HELP, i, r.get("wave_slot_mean", 0.0))
            for x, nb in enumerate(r["xcc_blocks"]):
                if nb:
                    add("gpu_probe_xcd_blocks", "Probe workgroups executed per XCD (liveness).", i, nb, {"xcd": str(x)})
                    add("gpu_probe_xcd_clock_mhz", "Effective shader clock per XCD measured in-kernel.", i,
                        r["xcc_clock_mhz"][x], {"xcd": str(x)})
                    add("gpu_probe_xcd_wave_slot_mean", SLOT_HELP, i, r["xcc_wave_slot"][x], {"xcd": str(x)})
        self.ex.set_extra("probe", series)

    def start(self):
        self._th = threading.Thread(target=self._loop, name="gpumon-probe", daemon=True)
        self._th.start()
        return self

    def _loop(self):
        while not self._stop.is_set():
            t0 = time.monotonic()
            try:
                self.step()
            except Exception:  # noqa: BLE001
                log.exception("probe step failed")
            self._stop.wait(max(0.0, self.every_s - (time.monotonic() - t0)))

    def stop(self):
        self._stop.set()
        if self._th:
            self._th.join(timeout=5)
        # drain in-flight launches before the Probe objects (and their pinned ring) go away
        for i, slot in list(self.pending.items()):
            self.probes[i].poll(slot, 2.0)
        self.ex.set_extra("probe", [])
