"""Native kubelet PodResources client (csrc/core/grpc_lite.cpp: HTTP/2 + gRPC + protobuf by hand)
against the in-process fake kubelet (a real grpcio server on a unix socket), and the exporter's
native poller that turns allocations into idle pod_gpu rows for the standalone binary."""

import os
import subprocess
import time
import urllib.request

import pytest

from oracles.attribution.fake_kubelet import FakeKubelet, FakePod
from gpumon.export import promtext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def kubelet(tmp_path):
    sock = str(tmp_path / "kubelet.sock")
    with FakeKubelet(podres_socket=sock) as k:
        k.pods = [FakePod("jupyter-e-0", "ml", "u1", containers={"nb": ("c1", ["0000:05:00.0", "0000:25:00.0"])}),
                  FakePod("train-q-1", "team", "u2", containers={"w": ("c2", ["0000:45:00.0"]), "side": ("c3", [])}),
                  FakePod("ghost", "x", "u3", containers={"g": ("c4", ["0000:ff:00.0"])})]
        yield sock, k


def test_client_lists_allocations(core, kubelet):
    sock, k = kubelet
    rows = core.podresources_list(sock)
    assert [(r["namespace"], r["pod"], r["container"], r["device_id"]) for r in rows] == [
        ("ml", "jupyter-e-0", "nb", "0000:05:00.0"), ("ml", "jupyter-e-0", "nb", "0000:25:00.0"),
        ("team", "train-q-1", "w", "0000:45:00.0"), ("x", "ghost", "g", "0000:ff:00.0")]
    assert {r["resource"] for r in rows} == {"amd.com/gpu"}
    assert core.podresources_list(sock, "nvidia.com/") == []
    assert k.calls["list"] == 2


def test_client_errors_are_reported(core, tmp_path):
    with pytest.raises(RuntimeError, match="connect"):
        core.podresources_list(str(tmp_path / "missing.sock"))


def test_parser_matches_python_protobuf(core):
    from oracles.attribution import proto as P

    r = P.ListPodResourcesResponse()
    pr = r.pod_resources.add(name="p", namespace="n")
    c = pr.containers.add(name="c")
    c.devices.add(resource_name="amd.com/gpu", device_ids=["a", "b"])
    c.devices.add(resource_name="example.com/nic", device_ids=["z"])
    assert core.parse_list_pod_resources(r.SerializeToString(), "amd.com/") == [
        ("n", "p", "c", "amd.com/gpu", "a"), ("n", "p", "c", "amd.com/gpu", "b")]
    with pytest.raises(RuntimeError):
        core.parse_list_pod_resources(b"\x0a\xff\x01", "")


def test_exporter_poller_builds_idle_rows(core, kubelet):
    sock, _ = kubelet
    ex = core.Exporter({"backend": "mock:gpus=4,mode=idle", "serve_http": False, "interval_s": 0,
                        "pod_resources_socket": sock, "pod_resources_refresh_s": 0.5, "host": "n1"})
    ex.start()
    try:
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpumon_podresources_up") == 1
        assert promtext.one(fam, "gpumon_podresources_unknown_devices") == 1  # 0000:ff:00.0
        alloc = promtext.values(fam, "pod_gpu_allocated", podname="jupyter-e-0")
        assert len(alloc) == 2
        assert promtext.one(fam, "gpumon_gpus", state="allocated") == 3
        assert promtext.one(fam, "gpumon_gpus", state="allocated_idle") == 3
    finally:
        ex.stop()


@pytest.mark.slow
def test_native_binary_uses_pod_resources(kubelet):
    sock, _ = kubelet
    subprocess.run(["make", "-C", ROOT, "core"], check=True, stdout=subprocess.DEVNULL)
    import socket as so

    with so.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.Popen([os.path.join(ROOT, "bin/gpumon-exporter"), "--backend", "mock:gpus=2,mode=idle",
                          "--interval", "0.2", "--listen", f"127.0.0.1:{port}", "--pod-resources", sock,
                          "--log-level", "error"], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        body = ""
        for _ in range(50):
            try:
                body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=2).read().decode()
                if "pod_gpu_allocated" in body:
                    break
            except OSError:
                pass
            time.sleep(0.1)
        fam = promtext.parse(body)
        assert promtext.one(fam, "gpumon_podresources_up") == 1
        assert len(promtext.values(fam, "pod_gpu_allocated")) == 2
    finally:
        p.terminate()
        p.wait(timeout=10)


from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=300, deadline=None)
@given(data=st.binary(max_size=256))
def test_parser_never_crashes_on_garbage(data):
    from gpumon import core as _core

    try:
        rows = _core().parse_list_pod_resources(data, "")
        assert isinstance(rows, list)
    except RuntimeError:
        pass


CID_A = "aa" * 32
CID_B = "bb" * 32


def _fake_proc(root, pid, cid):
    d = root / str(pid)
    d.mkdir(parents=True)
    (d / "stat").write_text(f"{pid} (train) S 1 1 1 0 -1 0 0 0 0 0 0 0 0 0 20 0 1 0 777 0 0\n")
    (d / "cgroup").write_text(f"0::/kubepods.slice/cri-containerd-{cid}.scope\n")


def test_native_cri_client(core, tmp_path):
    d = f"/tmp/gpumon-ncri-{os.getpid()}"
    os.makedirs(d, exist_ok=True)
    with FakeKubelet(cri_socket=f"{d}/cri.sock") as k:
        k.pods = [FakePod("jupyter-q-0", "research", "uid-b", labels={"team": "q"},
                          containers={"main": (CID_B, ["0000:25:00.0"])})]
        cs, sbs = core.cri_list(k.cri_socket)
    assert [c["id"] for c in cs] == [CID_B]
    assert cs[0]["labels"]["io.kubernetes.pod.name"] == "jupyter-q-0"
    assert sbs[0]["name"] == "jupyter-q-0" and sbs[0]["namespace"] == "research" and sbs[0]["uid"] == "uid-b"
    assert sbs[0]["labels"]["team"] == "q"


def test_native_control_plane_end_to_end(core, tmp_path):
    """Same scenario as test_control_plane.test_plane_end_to_end, with no Python control plane:
    the exporter's own CRI + PodResources pollers (what bin/gpumon-exporter runs)."""
    d = f"/tmp/gpumon-nkl-{os.getpid()}"
    os.makedirs(d, exist_ok=True)
    with FakeKubelet(podres_socket=f"{d}/kubelet.sock", cri_socket=f"{d}/cri.sock") as k:
        k.pods = [
            FakePod("turing-gpu-notebook-alice-1-2", "ml", "uid-a", labels={"mlgpu": "mlgpu"},
                    containers={"nb": (CID_A, ["0000:05:00.0"])}),
            FakePod("jupyter-q-0", "research", "uid-b", containers={"main": (CID_B, ["0000:25:00.0"])}),
        ]
        _fake_proc(tmp_path, 1000, CID_A)
        ex = core.Exporter({"backend": "mock:gpus=2", "serve_http": False, "interval_s": 0, "host": "n1",
                            "procfs_root": str(tmp_path), "cri_socket": k.cri_socket,
                            "pod_resources_socket": k.podres_socket})
        ex.start()
        try:
            ex.mock_set_procs([{"pid": 1000, "device": 0, "name": "python", "vram_bytes": 5 << 30}])
            ex.tick()
            rows = {(r["podname"], r["idle"]): r for r in ex.pod_rows()}
            active = rows[("turing-gpu-notebook-alice-1-2", False)]
            assert (active["namespace"], active["container"], active["user_name"], active["containerid"],
                    active["pid"]) == ("ml", "nb", "alice", CID_A[:12], "1000")
            idle = rows[("jupyter-q-0", True)]
            assert (idle["pid"], idle["user_name"], idle["dev"], idle["containerid"]) == ("-", "q", 1, CID_B[:12])
            fam = promtext.parse(ex.metrics_text())
            assert promtext.one(fam, "gpumon_cri_up") == 1 and promtext.one(fam, "gpumon_cri_containers") == 2
            assert promtext.one(fam, "gpumon_podresources_up") == 1
            assert promtext.one(fam, "gpumon_gpus", state="allocated_active") == 1
        finally:
            ex.stop()


def test_gpumon_monitor_native_mode(tmp_path):
    """`gpumon serve --control-plane native`: the Python monitor hands the sockets to the C++
    pollers instead of starting the grpcio control plane."""
    from gpumon.config import Config
    from gpumon.monitor import GpuMonitor

    d = f"/tmp/gpumon-nm-{os.getpid()}"
    os.makedirs(d, exist_ok=True)
    with FakeKubelet(podres_socket=f"{d}/kubelet.sock", cri_socket=f"{d}/cri.sock") as k:
        k.pods = [FakePod("jupyter-q-0", "research", "uid-b", containers={"main": (CID_B, ["0000:25:00.0"])})]
        cfg = Config(backend="mock:gpus=2,mode=idle", interval=0, listen="127.0.0.1:0", control_plane="native",
                     pod_resources_socket=k.podres_socket, cri_socket=k.cri_socket, log_level="warn")
        with GpuMonitor(cfg) as mon:
            assert mon.control_plane_mode == "native" and mon.plane is None
            mon.ex.tick()
            idle = [r for r in mon.ex.pod_rows() if r["idle"]]
            assert [(r["podname"], r["dev"], r["containerid"]) for r in idle] == [("jupyter-q-0", 1, CID_B[:12])]


_txt = st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=12)
_labels = st.dictionaries(_txt, _txt, max_size=4)


@settings(max_examples=150, deadline=None)
@given(cs=st.lists(st.tuples(_txt, _txt, _txt, _labels, _labels, st.integers(0, 3), st.integers(0, 2 ** 62)),
                   max_size=5),
       unknown=st.booleans())
def test_cri_container_parser_matches_protobuf(cs, unknown):
    """The hand-written CRI decoder (grpc_lite.cpp parse_cri_containers) against python-protobuf's
    encoding of the same ListContainersResponse: every field the exporter reads, fields it skips
    (image, state, created_at), and an unknown top-level field (a newer runtime's)."""
    from gpumon import core as _core
    from oracles.attribution import proto as P

    r = P.ListContainersResponse()
    for cid, sb, name, labels, ann, state, created in cs:
        c = r.containers.add(id=cid, pod_sandbox_id=sb, image_ref="sha256:x", state=state, created_at=created)
        c.metadata.name = name
        c.metadata.attempt = 2
        c.image.image = "rocm/pytorch"
        c.labels.update(labels)
        c.annotations.update(ann)
    raw = r.SerializeToString() + (b"\x78\x01\x82\x01\x02hi" if unknown else b"")
    got = _core().parse_cri_containers(raw)
    assert got == [(cid, sb, name, labels, ann) for cid, sb, name, labels, ann, _, _ in cs]


@settings(max_examples=150, deadline=None)
@given(ss=st.lists(st.tuples(_txt, _txt, _txt, _txt, _labels, _labels), max_size=5))
def test_cri_sandbox_parser_matches_protobuf(ss):
    from gpumon import core as _core
    from oracles.attribution import proto as P

    r = P.ListPodSandboxResponse()
    for sid, name, uid, ns, labels, ann in ss:
        i = r.items.add(id=sid, state=0, created_at=5, runtime_handler="runc")
        i.metadata.name, i.metadata.uid, i.metadata.namespace, i.metadata.attempt = name, uid, ns, 1
        i.labels.update(labels)
        i.annotations.update(ann)
    assert _core().parse_cri_sandboxes(r.SerializeToString()) == [tuple(x) for x in ss]


@settings(max_examples=300, deadline=None)
@given(data=st.binary(max_size=256))
def test_cri_parsers_never_crash_on_garbage(data):
    from gpumon import core as _core

    for fn in (_core().parse_cri_containers, _core().parse_cri_sandboxes):
        try:
            assert isinstance(fn(data), list)
        except RuntimeError:
            pass
