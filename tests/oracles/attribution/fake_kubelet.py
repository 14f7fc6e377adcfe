"""In-process fake kubelet PodResources + CRI runtime gRPC servers (unix sockets).

Used by the tests and by ``gpumon demo`` to exercise the whole attribution path (CRI labels ->
container meta, PodResources -> idle-allocation rows) without a cluster. The reference had no
fakes or tests of any kind.
"""

from __future__ import annotations

from concurrent import futures
from dataclasses import dataclass, field
from typing import Dict, List

import grpc

from . import proto as P


@dataclass
class FakePod:
    name: str
    namespace: str
    uid: str
    labels: Dict[str, str] = field(default_factory=dict)
    annotations: Dict[str, str] = field(default_factory=dict)
    # container name -> (container id, device ids)
    containers: Dict[str, tuple] = field(default_factory=dict)
    # container name -> DRA claimed devices [(driver, device name, cdi name)] (one claim per container)
    claims: Dict[str, List[tuple]] = field(default_factory=dict)


class FakeKubelet:
    def __init__(self, podres_socket: str = "", cri_socket: str = "", resource_name: str = "amd.com/gpu",
                 cri_api: str = "runtime.v1"):
        self.podres_socket = podres_socket
        self.cri_socket = cri_socket
        self.resource_name = resource_name
        self.pods: List[FakePod] = []
        self.allocatable: List[str] = []
        self.calls = {"list": 0, "containers": 0, "sandboxes": 0}
        self.fail_cri = False
        # (grpc.StatusCode, message) the PodResources List() answers with instead of a response
        self.podres_error = None
        self.cri_api = cri_api  # "runtime.v1" | "runtime.v1alpha2" (containerd < 1.7)
        self._servers = []

    # ---------------------------------------------------------------- handlers
    def _list(self, req, ctx):
        self.calls["list"] += 1
        if self.podres_error is not None:
            ctx.abort(*self.podres_error)
        r = P.ListPodResourcesResponse()
        for p in self.pods:
            pr = r.pod_resources.add(name=p.name, namespace=p.namespace)
            for cname, (_cid, devs) in p.containers.items():
                c = pr.containers.add(name=cname)
                if devs:
                    c.devices.add(resource_name=self.resource_name, device_ids=list(devs))
                if p.claims.get(cname):
                    dr = c.dynamic_resources.add(claim_name=f"{p.name}-{cname}-gpu", claim_namespace=p.namespace)
                    for driver, dev, cdi in p.claims[cname]:
                        cr = dr.claim_resources.add(driver_name=driver, pool_name="node-a", device_name=dev)
                        if cdi:
                            cr.cdi_devices.add(name=cdi)
        return r

    def _allocatable(self, req, ctx):
        r = P.AllocatableResourcesResponse()
        if self.allocatable:
            r.devices.add(resource_name=self.resource_name, device_ids=list(self.allocatable))
        return r

    def _version(self, req, ctx):
        return P.VersionResponse(version="0.1.0", runtime_name="fake-containerd", runtime_version="1.7.0",
                                 runtime_api_version="v1")

    def _containers(self, req, ctx):
        self.calls["containers"] += 1
        if self.fail_cri:
            ctx.abort(grpc.StatusCode.UNAVAILABLE, "injected failure")
        r = P.ListContainersResponse()
        for p in self.pods:
            for cname, (cid, _devs) in p.containers.items():
                c = r.containers.add(id=cid, pod_sandbox_id="sb-" + p.uid, state=P.CONTAINER_RUNNING)
                c.metadata.name = cname
                c.labels.update({
                    "io.kubernetes.pod.name": p.name,
                    "io.kubernetes.pod.namespace": p.namespace,
                    "io.kubernetes.pod.uid": p.uid,
                    "io.kubernetes.container.name": cname,
                })
        return r

    def _sandboxes(self, req, ctx):
        self.calls["sandboxes"] += 1
        r = P.ListPodSandboxResponse()
        for p in self.pods:
            s = r.items.add(id="sb-" + p.uid, state=P.SANDBOX_READY)
            s.metadata.name = p.name
            s.metadata.uid = p.uid
            s.metadata.namespace = p.namespace
            s.labels.update(p.labels)
            s.annotations.update(p.annotations)
        return r

    # ---------------------------------------------------------------- lifecycle
    def start(self):
        def h(fn, req_cls, resp_cls):
            return grpc.unary_unary_rpc_method_handler(fn, request_deserializer=req_cls.FromString,
                                                       response_serializer=resp_cls.SerializeToString)

        if self.podres_socket:
            s = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
            s.add_generic_rpc_handlers((grpc.method_handlers_generic_handler("v1.PodResourcesLister", {
                "List": h(self._list, P.ListPodResourcesRequest, P.ListPodResourcesResponse),
                "GetAllocatableResources": h(self._allocatable, P.AllocatableResourcesRequest,
                                             P.AllocatableResourcesResponse),
            }),))
            s.add_insecure_port("unix://" + self.podres_socket)
            s.start()
            self._servers.append(s)
        if self.cri_socket:
            s = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
            s.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{self.cri_api}.RuntimeService", {
                "Version": h(self._version, P.VersionRequest, P.VersionResponse),
                "ListContainers": h(self._containers, P.ListContainersRequest, P.ListContainersResponse),
                "ListPodSandbox": h(self._sandboxes, P.ListPodSandboxRequest, P.ListPodSandboxResponse),
            }),))
            s.add_insecure_port("unix://" + self.cri_socket)
            s.start()
            self._servers.append(s)
        return self

    def stop(self):
        for s in self._servers:
            s.stop(grace=None)
        self._servers.clear()

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()
