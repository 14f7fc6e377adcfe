"""Dynamic Resource Allocation (DRA): GPUs claimed through a DRA driver (default ``gpu.amd.com``)
appear in kubelet PodResources under ContainerResources.dynamic_resources instead of
ContainerDevices. Both control planes (Python grpcio client and the native grpc_lite poller) turn
them into allocations, and both device matchers accept the DRA id forms (CDI names, ``gpu-N``,
dashed PCI addresses). The AMD DRA driver's exact device naming is not pinned by any fixture in the
reference (which predates DRA): parity unpinned; the accepted forms are documented in
tests/oracles/attribution/plane.py."""


import pytest

from oracles.attribution import proto as P
from oracles.attribution.fake_kubelet import FakeKubelet, FakePod
from oracles.attribution.plane import match_device_id
from gpumon.export import promtext

STATICS = [{"index": i, "hip_id": i, "bdf": f"0000:{0x05 + 0x20 * i:02x}:00.0", "uuid": f"u{i}", "drm_card": i,
            "drm_render": 128 + i} for i in range(4)]


@pytest.mark.parametrize("dev_id,idx", [
    ("gpu-2", 2), ("amd.com/gpu=gpu-1", 1), ("gpu-0000-25-00-0", 1), ("pci-0000-45-00-0", 2), ("0000-65-00-0", 3),
    ("amd.com/gpu=0000:05:00.0", 0), ("gpu-9", -1), ("gpu-0000-99-00-0", -1), ("gpu-u3", 3), ("gpu-", -1),
    ("0000:25:00.0", 1), ("3", 3), ("renderD129", 1)])
def test_python_and_native_matchers_agree(core, dev_id, idx):
    assert match_device_id(dev_id, STATICS) == idx
    assert core.match_device_id(dev_id, STATICS) == idx


def test_native_parser_reads_dynamic_resources(core):
    r = P.ListPodResourcesResponse()
    pr = r.pod_resources.add(name="train-0", namespace="ml")
    c = pr.containers.add(name="w")
    c.devices.add(resource_name="amd.com/gpu", device_ids=["0000:05:00.0"])
    dr = c.dynamic_resources.add(claim_name="gpus", claim_namespace="ml")
    dr.claim_resources.add(driver_name="gpu.amd.com", pool_name="n1", device_name="gpu-1")
    cr = dr.claim_resources.add(driver_name="gpu.amd.com", pool_name="n1")  # no device name: CDI id
    cr.cdi_devices.add(name="amd.com/gpu=gpu-2")
    dr.claim_resources.add(driver_name="nic.example.com", device_name="eth-0")
    rows = core.parse_list_pod_resources(r.SerializeToString(), "amd.com/", ["gpu.amd.com"])
    assert rows == [("ml", "train-0", "w", "gpu.amd.com", "gpu-1"), ("ml", "train-0", "w", "gpu.amd.com",
                                                                      "amd.com/gpu=gpu-2"),
                    ("ml", "train-0", "w", "amd.com/gpu", "0000:05:00.0")]
    assert len(core.parse_list_pod_resources(r.SerializeToString(), "amd.com/")) == 1  # DRA off


@pytest.fixture
def kubelet(tmp_path):
    sock = str(tmp_path / "kubelet.sock")
    with FakeKubelet(podres_socket=sock) as k:
        k.pods = [FakePod("dp-0", "ml", "u1", containers={"nb": ("c1", ["0000:05:00.0"])}),
                  FakePod("dra-0", "team", "u2", containers={"w": ("c2", [])},
                          claims={"w": [("gpu.amd.com", "gpu-1", ""), ("gpu.amd.com", "", "amd.com/gpu=gpu-2")]}),
                  FakePod("other", "x", "u3", containers={"g": ("c3", [])},
                          claims={"g": [("nic.example.com", "eth-0", "")]})]
        yield sock, k


def test_python_client_lists_dra_claims(kubelet):
    from oracles.attribution.clients import PodResourcesClient

    sock, _ = kubelet
    cl = PodResourcesClient(sock)
    try:
        got = [(a.pod_name, a.resource_name, a.device_ids, a.claim) for a in cl.list(["amd.com/gpu"], ["gpu.amd.com"])]
    finally:
        cl.close()
    assert got == [("dp-0", "amd.com/gpu", ["0000:05:00.0"], ""),
                   ("dra-0", "gpu.amd.com", ["gpu-1"], "team/dra-0-w-gpu"),
                   ("dra-0", "gpu.amd.com", ["amd.com/gpu=gpu-2"], "team/dra-0-w-gpu")]


def _check_idle_rows(text):
    fam = promtext.parse(text)
    assert promtext.one(fam, "gpumon_gpus", state="allocated") == 3
    dra = promtext.values(fam, "pod_gpu_allocated", podname="dra-0")
    assert len(dra) == 2
    assert {s[1]["gpu_id"] for s in fam["pod_gpu_allocated"]["samples"] if s[1]["podname"] == "dra-0"} == {"1", "2"}


def test_native_poller_counts_dra_allocations(core, kubelet):
    sock, _ = kubelet
    ex = core.Exporter({"backend": "mock:gpus=4,mode=idle", "serve_http": False, "interval_s": 0,
                        "pod_resources_socket": sock, "pod_resources_refresh_s": 0.5, "host": "n1"})
    ex.start()
    try:
        ex.tick()
        _check_idle_rows(ex.metrics_text())
    finally:
        ex.stop()


def test_python_plane_counts_dra_allocations(kubelet, mock_exporter):
    from oracles.attribution.clients import PodResourcesClient
    from oracles.attribution.plane import ControlPlane
    from gpumon.config import Config

    sock, _ = kubelet
    ex = mock_exporter(backend="mock:gpus=4,mode=idle")
    plane = ControlPlane(ex, Config(), cri=None, podres=PodResourcesClient(sock))
    plane.refresh_once()
    ex.tick()
    _check_idle_rows(ex.metrics_text())
