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
import os
from typing import Optional

from ._native import core
from .config import Config

log = logging.getLogger("gpumon")

_LEVELS = {"debug": 0, "info": 1, "warn": 2, "warning": 2, "error": 3, "off": 4}


# well-known CRI sockets (the native pollers take the first that exists)
_CRI_SOCKETS = ("/run/containerd/containerd.sock", "/var/run/containerd/containerd.sock", "/var/run/crio/crio.sock",
                "/run/crio/crio.sock", "/var/run/cri-dockerd.sock", "/var/run/dockershim.sock")


class GpuMonitor:
    def __init__(self, cfg: Optional[Config] = None, control_plane: bool = True):
        self.cfg = cfg or Config()
        self._core = core()
        self._core.set_log_level(_LEVELS.get(self.cfg.log_level.lower(), 1))
        core_cfg = self.cfg.to_core()
        mode = self.cfg.control_plane if control_plane else "off"
        if mode not in ("native", "off"):
            # control_plane: python selected the grpcio test oracle of earlier releases (now under
            # tests/oracles, not shipped): the native pollers do the same work
            log.warning("control_plane=%s is not available in the exporter: using native", mode)
            mode = "native"
        if mode == "native":
            # the exporter's own C++ pollers (csrc/core/grpc_lite.cpp) -- same as bin/gpumon-exporter
            if self.cfg.pod_resources_socket not in ("", "none") and os.path.exists(self.cfg.pod_resources_socket):
                core_cfg["pod_resources_socket"] = self.cfg.pod_resources_socket
            # "" = autodetect, "none" = no CRI source (same rule as the native binary's options)
            cri = self.cfg.cri_socket or next((p for p in _CRI_SOCKETS if os.path.exists(p)), "")
            if cri and cri != "none":
                core_cfg["cri_socket"] = cri[len("unix://"):] if cri.startswith("unix://") else cri
            if self.cfg.docker_socket:  # opt-in: never autodetected (root-equivalent socket)
                d = self.cfg.docker_socket
                core_cfg["docker_socket"] = d[len("unix://"):] if d.startswith("unix://") else d
            if self.cfg.pod_log_root:
                core_cfg["pod_log_root"] = self.cfg.pod_log_root
            if self.cfg.device_checkpoint:
                core_cfg["device_checkpoint"] = self.cfg.device_checkpoint
            core_cfg["pod_resources_refresh_s"] = float(self.cfg.metadata_refresh)
            if self.cfg.resource_names:
                core_cfg["pod_resources_prefix"] = self.cfg.resource_names[0]
            core_cfg["pod_resources_dra_drivers"] = list(self.cfg.dra_drivers)
        self.control_plane_mode = mode
        self.ex = self._core.Exporter(core_cfg)
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
        period = max(self.cfg.interval, 0.1)
        # C++ threads over the same plugins the standalone binary dlopen()s (csrc/core/ondevice.h);
        # PMC initialises before the probe (rocprofiler must register before HIP brings HSA up).
        self.ondevice = self._core.OnDevice(self.ex, {
            "plugin_dir": self.cfg.plugin_dir, "pmc": bool(self.cfg.enable_pmc),
            "pmc_counters": list(self.cfg.pmc_counters), "pmc_every_s": period, "pmc_mode": self.cfg.pmc_mode,
            "ondevice_isolate": self.cfg.ondevice_isolate, "helper_retry_s": float(self.cfg.helper_retry),
            "probe": bool(self.cfg.enable_probe), "probe_every_s": period * self.cfg.probe_every})
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
        host = self.cfg.listen_addr
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
