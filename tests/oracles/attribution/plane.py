"""Control plane: keeps the C++ core's container metadata and GPU allocation tables fresh.

Runs beside the native sampler (never on its hot path). Every ``metadata_refresh`` seconds it
  1. lists running containers + pod sandboxes from the CRI runtime and pushes
     ``container_id -> {pod, namespace, container, uid, labels}`` to the core
     (reference: ``docker inspect`` labels, /root/reference/gpu.py:184,192-195);
  2. lists kubelet PodResources allocations of ``amd.com/gpu`` and pushes
     ``(pod, container) -> gpu index`` so the core can emit idle-allocation rows
     (reference: ``docker exec ... nvidia-smi -L``, gpu.py:220-253).
Failures are isolated per source and exported as ``gpumon_control_plane_up{source}``.
"""

from __future__ import annotations

import logging
import re
import threading
import time
from typing import Dict, List, Optional

from .clients import CRIClient, PodResourcesClient, detect_cri_socket

log = logging.getLogger("gpumon.plane")


def normalize_id(s: str) -> str:
    return s.strip().lower()


_DASHED_BDF = re.compile(r"^(?:gpu-|pci-)?([0-9a-f]{4})-([0-9a-f]{2})-([0-9a-f]{2})-([0-7])$")


def match_device_id(dev_id: str, statics: List[dict]) -> int:
    """Map a device-plugin device ID to an exporter device index (-1 if unknown).

    Accepts PCI addresses with or without domain (AMD k8s-device-plugin uses the PCI bus id),
    amdsmi UUIDs, HIP uuids (``GPU-...``), plain hip ids, ``cardN`` / ``renderDN``, and the DRA
    forms: a CDI name (``amd.com/gpu=gpu-0``: the part after ``=``), ``gpu-N`` (hip id N) and
    dashed PCI addresses (``gpu-0000-26-00-0`` / ``0000-26-00-0``). Same rules as the C++
    ``match_device_id`` (csrc/core/control_plane.cpp).
    """
    d = normalize_id(dev_id)
    if "=" in d:
        d = d.split("=", 1)[1]
    m = _DASHED_BDF.match(d)
    if m:
        d = "%s:%s:%s.%s" % m.groups()
    elif d.startswith("gpu-") and d[4:].isdigit():
        d = d[4:]
    if not d:
        return -1
    for s in statics:
        bdf = (s.get("bdf") or "").lower()
        if bdf and (d == bdf or (":" in d and bdf.endswith(d)) or d == bdf.split(":", 1)[-1]):
            return s["index"]
        uuid = (s.get("uuid") or "").lower()
        if uuid and (d == uuid or d == "gpu-" + uuid):
            return s["index"]
    for s in statics:
        if d.isdigit() and int(d) == s.get("hip_id"):
            return s["index"]
        if d.startswith("card") and d[4:].isdigit() and int(d[4:]) == s.get("drm_card"):
            return s["index"]
        if d.startswith("renderd") and d[7:].isdigit() and int(d[7:]) == s.get("drm_render"):
            return s["index"]
    return -1


class ControlPlane:
    def __init__(self, exporter, cfg, cri: Optional[CRIClient] = None,
                 podres: Optional[PodResourcesClient] = None):
        self.ex = exporter
        self.cfg = cfg
        self.cri = cri
        self.podres = podres
        if self.cri is None:
            sock = detect_cri_socket(cfg.cri_socket)
            if sock:
                self.cri = CRIClient(sock)
        if self.podres is None and cfg.pod_resources_socket:
            import os

            if os.path.exists(cfg.pod_resources_socket):
                self.podres = PodResourcesClient(cfg.pod_resources_socket)
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None
        self.status: Dict[str, dict] = {}
        self.refreshes = 0

    @property
    def enabled(self) -> bool:
        return self.cri is not None or self.podres is not None

    # ------------------------------------------------------------------ one refresh
    def refresh_once(self) -> dict:
        metas: List[dict] = []
        by_pod_container: Dict[tuple, dict] = {}
        if self.cri is not None:
            t0 = time.perf_counter()
            try:
                sandboxes = {s.id: s for s in self.cri.sandboxes()}
                for c in self.cri.containers():
                    sb = sandboxes.get(c.pod_sandbox_id)
                    labels: Dict[str, str] = {}
                    if sb is not None:
                        labels.update(sb.annotations)
                        labels.update(sb.labels)
                    labels.update(c.annotations)
                    labels.update(c.labels)
                    m = {
                        "container_id": c.id,
                        "container_name": c.labels.get("io.kubernetes.container.name") or c.name,
                        "pod_name": c.labels.get("io.kubernetes.pod.name") or (sb.name if sb else ""),
                        "pod_namespace": c.labels.get("io.kubernetes.pod.namespace") or (sb.namespace if sb else ""),
                        "pod_uid": c.labels.get("io.kubernetes.pod.uid") or (sb.uid if sb else ""),
                        "labels": labels,
                    }
                    metas.append(m)
                    by_pod_container[(m["pod_namespace"], m["pod_name"], m["container_name"])] = m
                self.ex.set_container_meta(metas)
                self.status["cri"] = {"up": 1, "containers": len(metas), "seconds": time.perf_counter() - t0}
            except Exception as e:  # noqa: BLE001 - isolate source failures
                self.status["cri"] = {"up": 0, "error": str(e)[:200]}
                log.warning("CRI refresh failed: %s", e)
        allocs: List[dict] = []
        if self.podres is not None:
            t0 = time.perf_counter()
            try:
                statics = self.ex.statics()
                unknown = 0
                for a in self.podres.list(self.cfg.resource_names, self.cfg.dra_drivers):
                    meta = by_pod_container.get((a.pod_namespace, a.pod_name, a.container_name), {})
                    for did in a.device_ids:
                        idx = match_device_id(did, statics)
                        if idx < 0:
                            unknown += 1
                            continue
                        allocs.append({
                            "pod_namespace": a.pod_namespace,
                            "pod_name": a.pod_name,
                            "container_name": a.container_name,
                            "container_id": meta.get("container_id", ""),
                            "pod_uid": meta.get("pod_uid", ""),
                            "gpu_index": idx,
                            "labels": meta.get("labels", {}),
                        })
                self.ex.set_allocations(allocs)
                self.status["podresources"] = {"up": 1, "allocations": len(allocs), "unknown_devices": unknown,
                                               "seconds": time.perf_counter() - t0}
            except Exception as e:  # noqa: BLE001
                self.status["podresources"] = {"up": 0, "error": str(e)[:200]}
                log.warning("PodResources refresh failed: %s", e)
        self.refreshes += 1
        self._export_status()
        return {"metas": len(metas), "allocations": len(allocs), "status": dict(self.status)}

    def _export_status(self):
        series = []
        for src, st in self.status.items():
            series.append({"name": "gpumon_control_plane_up", "help": "1 if the last metadata refresh from this source succeeded.",
                           "labels": {"source": src}, "value": float(st.get("up", 0))})
            if "seconds" in st:
                series.append({"name": "gpumon_control_plane_refresh_seconds", "help": "Duration of the last metadata refresh.",
                               "labels": {"source": src}, "value": float(st["seconds"])})
        self.ex.set_extra("control_plane", series)

    # ------------------------------------------------------------------ thread
    def start(self):
        if not self.enabled:
            return self
        self.refresh_once()
        self._th = threading.Thread(target=self._loop, name="gpumon-control-plane", daemon=True)
        self._th.start()
        return self

    def _loop(self):
        while not self._stop.wait(self.cfg.metadata_refresh):
            try:
                self.refresh_once()
            except Exception:  # noqa: BLE001
                log.exception("control plane refresh crashed")

    def stop(self):
        self._stop.set()
        if self._th:
            self._th.join(timeout=5)
        for c in (self.cri, self.podres):
            if c is not None:
                c.close()
