"""gRPC clients for kubelet PodResources and the CRI runtime service (unix sockets).

Reference equivalents (/root/reference/gpu.py):
  * ``docker ps`` / ``docker stats`` / ``docker inspect`` (gpu.py:86-103,184,192): container list and
    the ``io.kubernetes.pod.*`` labels                           -> :class:`CRIClient`
  * ``docker exec <cid> nvidia-smi -L | cut ...`` (gpu.py:221-224): GPUs visible inside an idle
    container                                                       -> :class:`PodResourcesClient`
Both are read-only; no docker socket (root-equivalent) is needed.
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import grpc

from . import proto as P

DEFAULT_CRI_SOCKETS = (
    "/run/containerd/containerd.sock",
    "/var/run/containerd/containerd.sock",
    "/run/crio/crio.sock",
    "/var/run/crio/crio.sock",
    "/run/cri-dockerd.sock",
    "/var/run/cri-dockerd.sock",
    "/var/run/dockershim.sock",  # kubelet <= 1.23 with the docker runtime (dockershim serves CRI)
)


def _target(sock: str) -> str:
    if sock.startswith("unix:"):
        return sock
    return "unix://" + sock


def _unary(channel: grpc.Channel, method: str, req_cls, resp_cls):
    return channel.unary_unary(method, request_serializer=req_cls.SerializeToString,
                               response_deserializer=resp_cls.FromString)


@dataclass
class DeviceAllocation:
    pod_namespace: str
    pod_name: str
    container_name: str
    resource_name: str          # device-plugin resource, or the DRA driver name
    device_ids: List[str]
    claim: str = ""             # DRA: "<claim namespace>/<claim name>"


class PodResourcesClient:
    """kubelet ``v1.PodResourcesLister`` over ``/var/lib/kubelet/pod-resources/kubelet.sock``."""

    def __init__(self, socket_path: str, timeout_s: float = 5.0):
        self.socket_path = socket_path
        self.timeout_s = timeout_s
        self._ch = grpc.insecure_channel(_target(socket_path))
        self._list = _unary(self._ch, P.PODRESOURCES_LIST, P.ListPodResourcesRequest, P.ListPodResourcesResponse)
        self._alloc = _unary(self._ch, P.PODRESOURCES_ALLOCATABLE, P.AllocatableResourcesRequest,
                             P.AllocatableResourcesResponse)

    def list(self, resource_names: Optional[List[str]] = None,
             dra_drivers: Optional[List[str]] = None) -> List[DeviceAllocation]:
        """Device-plugin allocations of ``resource_names`` plus DRA claim devices whose driver is in
        ``dra_drivers`` (device id = the driver's device name, else its first CDI device)."""
        resp = self._list(P.ListPodResourcesRequest(), timeout=self.timeout_s)
        out = []
        for pod in resp.pod_resources:
            for c in pod.containers:
                for d in c.devices:
                    if resource_names and d.resource_name not in resource_names:
                        continue
                    out.append(DeviceAllocation(pod.namespace, pod.name, c.name, d.resource_name, list(d.device_ids)))
                if not dra_drivers:
                    continue
                for dr in c.dynamic_resources:
                    for cr in dr.claim_resources:
                        if cr.driver_name not in dra_drivers:
                            continue
                        dev = cr.device_name or (cr.cdi_devices[0].name if cr.cdi_devices else "")
                        if dev:
                            out.append(DeviceAllocation(pod.namespace, pod.name, c.name, cr.driver_name, [dev],
                                                        claim=f"{dr.claim_namespace}/{dr.claim_name}"))
        return out

    def allocatable(self, resource_names: Optional[List[str]] = None) -> List[str]:
        resp = self._alloc(P.AllocatableResourcesRequest(), timeout=self.timeout_s)
        ids = []
        for d in resp.devices:
            if resource_names and d.resource_name not in resource_names:
                continue
            ids.extend(d.device_ids)
        return ids

    def close(self):
        self._ch.close()


@dataclass
class ContainerInfo:
    id: str
    name: str
    pod_sandbox_id: str
    labels: Dict[str, str] = field(default_factory=dict)
    annotations: Dict[str, str] = field(default_factory=dict)


@dataclass
class SandboxInfo:
    id: str
    name: str
    uid: str
    namespace: str
    labels: Dict[str, str] = field(default_factory=dict)
    annotations: Dict[str, str] = field(default_factory=dict)


class CRIClient:
    """CRI ``runtime.v1.RuntimeService`` (containerd, cri-o, cri-dockerd)."""

    def __init__(self, socket_path: str, timeout_s: float = 5.0):
        self.socket_path = socket_path
        self.timeout_s = timeout_s
        self._ch = grpc.insecure_channel(_target(socket_path))
        self._version = _unary(self._ch, P.CRI_VERSION, P.VersionRequest, P.VersionResponse)
        self._lc = _unary(self._ch, P.CRI_LIST_CONTAINERS, P.ListContainersRequest, P.ListContainersResponse)
        self._ls = _unary(self._ch, P.CRI_LIST_SANDBOXES, P.ListPodSandboxRequest, P.ListPodSandboxResponse)

    def version(self) -> Dict[str, str]:
        r = self._version(P.VersionRequest(version="v1"), timeout=self.timeout_s)
        return {"runtime_name": r.runtime_name, "runtime_version": r.runtime_version,
                "runtime_api_version": r.runtime_api_version}

    def containers(self, running_only: bool = True) -> List[ContainerInfo]:
        req = P.ListContainersRequest()
        if running_only:
            req.filter.state.state = P.CONTAINER_RUNNING
        resp = self._lc(req, timeout=self.timeout_s)
        return [ContainerInfo(c.id, c.metadata.name, c.pod_sandbox_id, dict(c.labels), dict(c.annotations))
                for c in resp.containers]

    def sandboxes(self, ready_only: bool = True) -> List[SandboxInfo]:
        req = P.ListPodSandboxRequest()
        if ready_only:
            req.filter.state.state = P.SANDBOX_READY
        resp = self._ls(req, timeout=self.timeout_s)
        return [SandboxInfo(s.id, s.metadata.name, s.metadata.uid, s.metadata.namespace, dict(s.labels),
                            dict(s.annotations)) for s in resp.items]

    def close(self):
        self._ch.close()


def detect_cri_socket(explicit: str = "") -> str:
    if explicit:
        return explicit
    for p in DEFAULT_CRI_SOCKETS:
        if os.path.exists(p):
            return p
    return ""
