"""Protobuf message classes for the two kubelet-side gRPC APIs the control plane talks to.

There is no ``protoc`` / grpcio-tools in the image, so the descriptors are declared here with
``descriptor_pb2`` (field numbers and types follow the upstream .proto files):

* ``k8s.io/kubelet/pkg/apis/podresources/v1/api.proto`` — service ``v1.PodResourcesLister``
  (``List``, ``GetAllocatableResources``, ``Get``): which pod/container holds which device IDs.
  This replaces the reference's ``docker exec <cid> nvidia-smi -L`` probe for allocated-but-idle
  GPUs (/root/reference/gpu.py:220-224).
* ``k8s.io/cri-api/pkg/apis/runtime/v1/api.proto`` — service ``runtime.v1.RuntimeService``
  (``ListContainers``, ``ListPodSandbox``, ``Version``): container id -> labels, the
  ``io.kubernetes.pod.name`` / ``io.kubernetes.pod.namespace`` labels the reference read through
  ``docker inspect`` (gpu.py:86-88,184,192-195).

Only the fields the exporter needs are declared; unknown fields on the wire are skipped by the
protobuf runtime, so newer kubelets/runtimes stay compatible.
"""

from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
_pool = descriptor_pool.DescriptorPool()


def _msg(fdp, name, fields, nested=()):
    m = fdp.message_type.add()
    m.name = name
    for n in nested:
        m.nested_type.add().CopyFrom(n)
    for (fname, num, ftype, label, type_name) in fields:
        f = m.field.add()
        f.name = fname
        f.number = num
        f.type = ftype
        f.label = label
        if type_name:
            f.type_name = type_name
    return m


def _map_entry(name, value_type=F.TYPE_STRING):
    e = descriptor_pb2.DescriptorProto()
    e.name = name
    e.options.map_entry = True
    k = e.field.add()
    k.name, k.number, k.type, k.label = "key", 1, F.TYPE_STRING, F.LABEL_OPTIONAL
    v = e.field.add()
    v.name, v.number, v.type, v.label = "value", 2, value_type, F.LABEL_OPTIONAL
    return e


OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED
STR, I64, U32, I32, MSG, ENUM, BOOL = (F.TYPE_STRING, F.TYPE_INT64, F.TYPE_UINT32, F.TYPE_INT32,
                                       F.TYPE_MESSAGE, F.TYPE_ENUM, F.TYPE_BOOL)

# ------------------------------------------------------------------------------------------
# kubelet PodResources v1
# ------------------------------------------------------------------------------------------
_pr = descriptor_pb2.FileDescriptorProto()
_pr.name = "gpumon/podresources_v1.proto"
_pr.package = "v1"
_pr.syntax = "proto3"
_msg(_pr, "ListPodResourcesRequest", [])
_msg(_pr, "NUMANode", [("ID", 1, I64, OPT, None)])
_msg(_pr, "TopologyInfo", [("nodes", 1, MSG, REP, ".v1.NUMANode")])
_msg(_pr, "ContainerDevices", [
    ("resource_name", 1, STR, OPT, None),
    ("device_ids", 2, STR, REP, None),
    ("topology", 3, MSG, OPT, ".v1.TopologyInfo"),
])
_msg(_pr, "ContainerMemory", [
    ("memory_type", 1, STR, OPT, None),
    ("size", 2, F.TYPE_UINT64, OPT, None),
    ("topology", 3, MSG, OPT, ".v1.TopologyInfo"),
])
# Dynamic Resource Allocation (k8s >= 1.27 kubelet; GPUs claimed through a DRA driver such as
# gpu.amd.com instead of the amd.com/gpu device-plugin resource). class_name (1) is the 1.27-1.30
# field, dropped later; decoding ignores it either way.
_msg(_pr, "CDIDevice", [("name", 1, STR, OPT, None)])
_msg(_pr, "ClaimResource", [
    ("cdi_devices", 1, MSG, REP, ".v1.CDIDevice"),
    ("driver_name", 2, STR, OPT, None),
    ("pool_name", 3, STR, OPT, None),
    ("device_name", 4, STR, OPT, None),
])
_msg(_pr, "DynamicResource", [
    ("class_name", 1, STR, OPT, None),
    ("claim_name", 2, STR, OPT, None),
    ("claim_namespace", 3, STR, OPT, None),
    ("claim_resources", 4, MSG, REP, ".v1.ClaimResource"),
])
_msg(_pr, "ContainerResources", [
    ("name", 1, STR, OPT, None),
    ("devices", 2, MSG, REP, ".v1.ContainerDevices"),
    ("cpu_ids", 3, I64, REP, None),
    ("memory", 4, MSG, REP, ".v1.ContainerMemory"),
    ("dynamic_resources", 5, MSG, REP, ".v1.DynamicResource"),
])
_msg(_pr, "PodResources", [
    ("name", 1, STR, OPT, None),
    ("namespace", 2, STR, OPT, None),
    ("containers", 3, MSG, REP, ".v1.ContainerResources"),
])
_msg(_pr, "ListPodResourcesResponse", [("pod_resources", 1, MSG, REP, ".v1.PodResources")])
_msg(_pr, "AllocatableResourcesRequest", [])
_msg(_pr, "AllocatableResourcesResponse", [
    ("devices", 1, MSG, REP, ".v1.ContainerDevices"),
    ("cpu_ids", 2, I64, REP, None),
    ("memory", 3, MSG, REP, ".v1.ContainerMemory"),
])
_msg(_pr, "GetPodResourcesRequest", [("pod_name", 1, STR, OPT, None), ("pod_namespace", 2, STR, OPT, None)])
_msg(_pr, "GetPodResourcesResponse", [("pod_resources", 1, MSG, OPT, ".v1.PodResources")])
_pool.Add(_pr)

# ------------------------------------------------------------------------------------------
# CRI runtime v1 (subset)
# ------------------------------------------------------------------------------------------
_cri = descriptor_pb2.FileDescriptorProto()
_cri.name = "gpumon/cri_runtime_v1.proto"
_cri.package = "runtime.v1"
_cri.syntax = "proto3"
_e = _cri.enum_type.add()
_e.name = "ContainerState"
for i, n in enumerate(["CONTAINER_CREATED", "CONTAINER_RUNNING", "CONTAINER_EXITED", "CONTAINER_UNKNOWN"]):
    v = _e.value.add()
    v.name, v.number = n, i
_e2 = _cri.enum_type.add()
_e2.name = "PodSandboxState"
for i, n in enumerate(["SANDBOX_READY", "SANDBOX_NOTREADY"]):
    v = _e2.value.add()
    v.name, v.number = n, i
_msg(_cri, "VersionRequest", [("version", 1, STR, OPT, None)])
_msg(_cri, "VersionResponse", [
    ("version", 1, STR, OPT, None),
    ("runtime_name", 2, STR, OPT, None),
    ("runtime_version", 3, STR, OPT, None),
    ("runtime_api_version", 4, STR, OPT, None),
])
_msg(_cri, "ContainerMetadata", [("name", 1, STR, OPT, None), ("attempt", 2, U32, OPT, None)])
_msg(_cri, "ImageSpec", [("image", 1, STR, OPT, None)])
_msg(_cri, "ContainerStateValue", [("state", 1, ENUM, OPT, ".runtime.v1.ContainerState")])
_msg(_cri, "ContainerFilter", [
    ("id", 1, STR, OPT, None),
    ("state", 2, MSG, OPT, ".runtime.v1.ContainerStateValue"),
    ("pod_sandbox_id", 3, STR, OPT, None),
    ("label_selector", 4, MSG, REP, ".runtime.v1.ContainerFilter.LabelSelectorEntry"),
], nested=[_map_entry("LabelSelectorEntry")])
_msg(_cri, "ListContainersRequest", [("filter", 1, MSG, OPT, ".runtime.v1.ContainerFilter")])
_msg(_cri, "Container", [
    ("id", 1, STR, OPT, None),
    ("pod_sandbox_id", 2, STR, OPT, None),
    ("metadata", 3, MSG, OPT, ".runtime.v1.ContainerMetadata"),
    ("image", 4, MSG, OPT, ".runtime.v1.ImageSpec"),
    ("image_ref", 5, STR, OPT, None),
    ("state", 6, ENUM, OPT, ".runtime.v1.ContainerState"),
    ("created_at", 7, I64, OPT, None),
    ("labels", 8, MSG, REP, ".runtime.v1.Container.LabelsEntry"),
    ("annotations", 9, MSG, REP, ".runtime.v1.Container.AnnotationsEntry"),
], nested=[_map_entry("LabelsEntry"), _map_entry("AnnotationsEntry")])
_msg(_cri, "ListContainersResponse", [("containers", 1, MSG, REP, ".runtime.v1.Container")])
_msg(_cri, "PodSandboxMetadata", [
    ("name", 1, STR, OPT, None),
    ("uid", 2, STR, OPT, None),
    ("namespace", 3, STR, OPT, None),
    ("attempt", 4, U32, OPT, None),
])
_msg(_cri, "PodSandboxStateValue", [("state", 1, ENUM, OPT, ".runtime.v1.PodSandboxState")])
_msg(_cri, "PodSandboxFilter", [
    ("id", 1, STR, OPT, None),
    ("state", 2, MSG, OPT, ".runtime.v1.PodSandboxStateValue"),
    ("label_selector", 3, MSG, REP, ".runtime.v1.PodSandboxFilter.LabelSelectorEntry"),
], nested=[_map_entry("LabelSelectorEntry")])
_msg(_cri, "ListPodSandboxRequest", [("filter", 1, MSG, OPT, ".runtime.v1.PodSandboxFilter")])
_msg(_cri, "PodSandbox", [
    ("id", 1, STR, OPT, None),
    ("metadata", 2, MSG, OPT, ".runtime.v1.PodSandboxMetadata"),
    ("state", 3, ENUM, OPT, ".runtime.v1.PodSandboxState"),
    ("created_at", 4, I64, OPT, None),
    ("labels", 5, MSG, REP, ".runtime.v1.PodSandbox.LabelsEntry"),
    ("annotations", 6, MSG, REP, ".runtime.v1.PodSandbox.AnnotationsEntry"),
    ("runtime_handler", 7, STR, OPT, None),
], nested=[_map_entry("LabelsEntry"), _map_entry("AnnotationsEntry")])
_msg(_cri, "ListPodSandboxResponse", [("items", 1, MSG, REP, ".runtime.v1.PodSandbox")])
_pool.Add(_cri)


def _cls(full_name):
    return message_factory.GetMessageClass(_pool.FindMessageTypeByName(full_name))


# PodResources
ListPodResourcesRequest = _cls("v1.ListPodResourcesRequest")
ListPodResourcesResponse = _cls("v1.ListPodResourcesResponse")
PodResources = _cls("v1.PodResources")
ContainerResources = _cls("v1.ContainerResources")
ContainerDevices = _cls("v1.ContainerDevices")
AllocatableResourcesRequest = _cls("v1.AllocatableResourcesRequest")
AllocatableResourcesResponse = _cls("v1.AllocatableResourcesResponse")
GetPodResourcesRequest = _cls("v1.GetPodResourcesRequest")
GetPodResourcesResponse = _cls("v1.GetPodResourcesResponse")

# CRI
VersionRequest = _cls("runtime.v1.VersionRequest")
VersionResponse = _cls("runtime.v1.VersionResponse")
ListContainersRequest = _cls("runtime.v1.ListContainersRequest")
ListContainersResponse = _cls("runtime.v1.ListContainersResponse")
Container = _cls("runtime.v1.Container")
ContainerMetadata = _cls("runtime.v1.ContainerMetadata")
ListPodSandboxRequest = _cls("runtime.v1.ListPodSandboxRequest")
ListPodSandboxResponse = _cls("runtime.v1.ListPodSandboxResponse")
PodSandbox = _cls("runtime.v1.PodSandbox")
PodSandboxMetadata = _cls("runtime.v1.PodSandboxMetadata")

CONTAINER_RUNNING = 1
SANDBOX_READY = 0

PODRESOURCES_LIST = "/v1.PodResourcesLister/List"
PODRESOURCES_ALLOCATABLE = "/v1.PodResourcesLister/GetAllocatableResources"
PODRESOURCES_GET = "/v1.PodResourcesLister/Get"
CRI_VERSION = "/runtime.v1.RuntimeService/Version"
CRI_LIST_CONTAINERS = "/runtime.v1.RuntimeService/ListContainers"
CRI_LIST_SANDBOXES = "/runtime.v1.RuntimeService/ListPodSandbox"
