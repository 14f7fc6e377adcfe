"""Control plane against an in-process fake kubelet (PodResources) + fake CRI runtime over unix
sockets: container labels -> pod rows, allocations -> idle rows, failure isolation.

Reference equivalents: docker inspect labels (gpu.py:184-195) and `docker exec nvidia-smi -L`
(gpu.py:220-253). The reference could only be tested on a live cluster; here it runs on CPU.
"""

import os
import time

import pytest

from oracles.attribution.fake_kubelet import FakeKubelet, FakePod
from oracles.attribution.plane import ControlPlane, match_device_id
from gpumon.config import Config
from gpumon.export import promtext

CID_A = "aa" * 32
CID_B = "bb" * 32


@pytest.fixture
def kubelet(tmp_path):
    # unix socket paths must be short
    d = f"/tmp/gpumon-kl-{os.getpid()}-{time.monotonic_ns() % 100000}"
    os.makedirs(d, exist_ok=True)
    k = FakeKubelet(podres_socket=f"{d}/kubelet.sock", cri_socket=f"{d}/cri.sock").start()
    yield k
    k.stop()


def _statics():
    return [{"index": 0, "hip_id": 0, "bdf": "0000:05:00.0", "uuid": "u0", "drm_card": 0, "drm_render": 128},
            {"index": 1, "hip_id": 1, "bdf": "0000:25:00.0", "uuid": "u1", "drm_card": 1, "drm_render": 129}]


@pytest.mark.parametrize("dev_id,idx", [("0000:25:00.0", 1), ("25:00.0", 1), ("0000:05:00.0", 0), ("u1", 1),
                                        ("GPU-u0", 0), ("1", 1), ("card0", 0), ("renderD129", 1),
                                        ("0000:99:00.0", -1), ("", -1)])
def test_match_device_id(dev_id, idx):
    assert match_device_id(dev_id, _statics()) == idx


def _fake_proc(root, pid, cid):
    d = root / str(pid)
    d.mkdir(parents=True)
    (d / "stat").write_text(f"{pid} (train) S 1 1 1 0 -1 0 0 0 0 0 0 0 0 0 20 0 1 0 777 0 0\n")
    (d / "cgroup").write_text(f"0::/kubepods.slice/cri-containerd-{cid}.scope\n")


def test_plane_end_to_end(kubelet, mock_exporter, tmp_path):
    kubelet.pods = [
        FakePod("turing-gpu-notebook-alice-1-2", "ml", "uid-a", labels={"mlgpu": "mlgpu"},
                containers={"nb": (CID_A, ["0000:05:00.0"])}),
        FakePod("jupyter-q-0", "research", "uid-b", containers={"main": (CID_B, ["0000:25:00.0"])}),
    ]
    _fake_proc(tmp_path, 1000, CID_A)
    ex = mock_exporter(backend="mock:gpus=2", procfs_root=str(tmp_path))
    ex.mock_set_procs([{"pid": 1000, "device": 0, "name": "python", "vram_bytes": 5 << 30}])
    cfg = Config(cri_socket=kubelet.cri_socket, pod_resources_socket=kubelet.podres_socket)
    plane = ControlPlane(ex, cfg)
    assert plane.enabled
    summary = plane.refresh_once()
    assert summary["metas"] == 2 and summary["allocations"] == 2
    ex.tick()
    rows = {(r["podname"], r["idle"]): r for r in ex.pod_rows()}
    active = rows[("turing-gpu-notebook-alice-1-2", False)]
    assert (active["namespace"], active["container"], active["user_name"], active["containerid"], active["pid"]) == (
        "ml", "nb", "alice", CID_A[:12], "1000")
    idle = rows[("jupyter-q-0", True)]
    assert (idle["pid"], idle["user_name"], idle["dev"], idle["containerid"]) == ("-", "q", 1, CID_B[:12])
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpumon_control_plane_up", source="cri") == 1
    assert promtext.one(fam, "gpumon_control_plane_up", source="podresources") == 1
    assert promtext.one(fam, "gpumon_gpus", state="allocated") == 2
    assert promtext.one(fam, "gpumon_gpus", state="allocated_active") == 1
    plane.stop()


def test_plane_opt_in_uses_pod_labels(kubelet, mock_exporter, tmp_path):
    """Q13: the opt-in label is a POD label (sandbox labels via CRI), not an image/docker label."""
    kubelet.pods = [
        FakePod("jupyter-e-0", "ml", "uid-e", labels={"mlgpu": "mlgpu"}, containers={"c": (CID_A, ["0000:05:00.0"])}),
        FakePod("jupyter-w-0", "ml", "uid-w", labels={}, containers={"c": (CID_B, ["0000:25:00.0"])}),
    ]
    ex = mock_exporter(backend="mock:gpus=2", procfs_root=str(tmp_path), opt_in="mlgpu=mlgpu")
    plane = ControlPlane(ex, Config(cri_socket=kubelet.cri_socket, pod_resources_socket=kubelet.podres_socket))
    plane.refresh_once()
    ex.tick()
    assert [r["podname"] for r in ex.pod_rows()] == ["jupyter-e-0"]
    plane.stop()


def test_plane_isolates_source_failures(kubelet, mock_exporter, tmp_path):
    kubelet.pods = [FakePod("jupyter-q-0", "r", "uid-q", containers={"m": (CID_B, ["0000:25:00.0"])})]
    kubelet.fail_cri = True
    ex = mock_exporter(backend="mock:gpus=2", procfs_root=str(tmp_path))
    plane = ControlPlane(ex, Config(cri_socket=kubelet.cri_socket, pod_resources_socket=kubelet.podres_socket))
    s = plane.refresh_once()
    assert s["status"]["cri"]["up"] == 0
    assert s["status"]["podresources"]["up"] == 1
    ex.tick()
    rows = ex.pod_rows()
    assert len(rows) == 1 and rows[0]["idle"] and rows[0]["containerid"] == "-"
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpumon_control_plane_up", source="cri") == 0
    plane.stop()


def test_plane_background_refresh(kubelet, mock_exporter, tmp_path):
    ex = mock_exporter(backend="mock:gpus=2", procfs_root=str(tmp_path))
    plane = ControlPlane(ex, Config(cri_socket=kubelet.cri_socket, pod_resources_socket=kubelet.podres_socket,
                                    metadata_refresh=0.05)).start()
    try:
        kubelet.pods = [FakePod("jupyter-z-0", "ml", "uid-z", containers={"c": (CID_A, ["1"])})]
        deadline = time.time() + 5
        while time.time() < deadline and plane.refreshes < 3:
            time.sleep(0.02)
        ex.tick()
        assert [r["podname"] for r in ex.pod_rows()] == ["jupyter-z-0"]
    finally:
        plane.stop()


def test_cri_version_and_allocatable(kubelet):
    from oracles.attribution.clients import CRIClient, PodResourcesClient

    kubelet.allocatable = ["0000:05:00.0", "0000:25:00.0"]
    c = CRIClient(kubelet.cri_socket)
    assert c.version()["runtime_name"] == "fake-containerd"
    p = PodResourcesClient(kubelet.podres_socket)
    assert p.allocatable(["amd.com/gpu"]) == kubelet.allocatable
    c.close()
    p.close()


def test_pod_label_allowlist_on_pod_gpu_series(kubelet, mock_exporter, tmp_path):
    """Allowlisted pod labels (kube-state-metrics style) land on every pod_gpu_* series of the pod,
    active and idle rows, as label_<sanitised key>; other labels do not."""
    kubelet.pods = [
        FakePod("train-a-0", "ml", "uid-a", labels={"team": "vision", "app.kubernetes.io/name": "trainer",
                                                    "secret-ish": "no"},
                containers={"nb": (CID_A, ["0000:05:00.0"])}),
        FakePod("idle-b-0", "ml", "uid-b", labels={"team": "nlp"}, containers={"main": (CID_B, ["0000:25:00.0"])}),
    ]
    _fake_proc(tmp_path, 1000, CID_A)
    ex = mock_exporter(backend="mock:gpus=2", procfs_root=str(tmp_path),
                       label_allowlist=["team", "app.kubernetes.io/name", "missing"])
    ex.mock_set_procs([{"pid": 1000, "device": 0, "name": "python", "vram_bytes": 5 << 30}])
    plane = ControlPlane(ex, Config(cri_socket=kubelet.cri_socket, pod_resources_socket=kubelet.podres_socket))
    plane.refresh_once()
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    (active,) = [s for s in fam["pod_gpu_used_memory_bytes"]["samples"] if s[1]["podname"] == "train-a-0"]
    assert active[1]["label_team"] == "vision" and active[1]["label_app_kubernetes_io_name"] == "trainer"
    assert "label_secret_ish" not in active[1] and "label_missing" not in active[1]
    (idle,) = [s for s in fam["pod_gpu_allocated"]["samples"] if s[1]["podname"] == "idle-b-0"]
    assert idle[1]["label_team"] == "nlp" and idle[1]["state"] == "idle"
    plane.stop()
