"""High-level Python handle over the native exporter + control plane + optional probe/PMC plugins.

    from gpumon.config import Config
    from gpumon.monitor import GpuMonitor
    with GpuMonitor(Config(backend="mock:gpus=8", listen="127.0.0.1:0")) as mon:
        print(mon.url, mon.metrics()[:200])

Replaces the reference's process entrypoint (/root/reference/gpu.py:258-267): instead of a
`while 1: main(); sleep(10)` loop that crashes on the first exception, the native sampler runs
on its own thread with per-GPU error isolation, and this object only wires the pieces together.
"""

from __future__ import annotations

import logging
from typing import Optional

from ._native import core
from .config import Config

log = logging.getLogger("gpumon")


class GpuMonitor:
    def __init__(self, cfg: Optional[Config] = None, control_plane: bool = True):
        self.cfg = cfg or Config()
        self._core = core()
        # the native options resolve everything: listen address, host fallback, the kubelet /
        # CRI / Docker / log-tree sources and their autodetect (csrc/core/options.cpp), exactly as
        # bin/gpumon-exporter does -- control_plane=False starts none of those pollers
        self.options = self.cfg.finalized(control_plane=control_plane)
        self._core.set_log_level(self.options.log_level_value)
        self.control_plane_mode = "native" if control_plane and self.cfg.control_plane == "native" else "off"
        self.ex = self._core.Exporter(self.options)
        self.plane = None      # kept for callers that check it: the control plane is in the core
        self.ondevice = None   # _core.OnDevice: PMC / probe samplers
        self.start_error = ""

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "GpuMonitor":
        # the on-device samplers first: the PMC helper process is spawned before anything in this
        # process touches the GPU; the samplers pick the devices up once the backend lists them
        if self.cfg.enable_pmc or self.cfg.enable_probe:
            self._start_ondevice()
        self.start_error = self.ex.start()
        if self.start_error:
            log.warning("backend not ready yet (will retry): %s", self.start_error)
        return self

    def _start_ondevice(self) -> None:
        # C++ threads over the same plugins the standalone binary dlopen()s (csrc/core/ondevice.h),
        # configured by the same finalized options (cadence from interval / probe_every);
        # PMC initialises before the probe (rocprofiler must register before HIP brings HSA up).
        self.ondevice = self._core.OnDevice(self.ex, self.options)
        self.ondevice.start()

    def step_ondevice(self) -> None:
        """One synchronous PMC / probe step (so a one-shot sample carries their series)."""
        if self.ondevice is not None:
            self.ondevice.step()

    def stop(self) -> None:
        for p in (self.ondevice,):
            if p is not None:
                try:
                    p.stop()
                except Exception:  # noqa: BLE001
                    log.exception("plugin stop failed")
        self.ex.stop()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ------------------------------------------------------------------ accessors
    @property
    def port(self) -> int:
        return self.ex.port

    @property
    def url(self) -> str:
        host = self.options.listen_addr
        if host in ("0.0.0.0", "", "::"):
            host = "127.0.0.1"  # the wildcard takes IPv4 loopback in both forms (dual-stack [::])
        elif ":" in host:
            host = f"[{host}]"
        scheme = "https" if self.cfg.tls_cert_file else "http"
        return f"{scheme}://{host}:{self.port}/metrics"

    def metrics(self) -> str:
        return self.ex.metrics_text()

    def tick(self) -> dict:
        return self.ex.tick()

    def wait_ticks(self, n: int = 1, timeout_s: float = 30.0) -> bool:
        return self.ex.wait_for_seq(self.ex.seq + n, timeout_s)
