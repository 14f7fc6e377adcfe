"""Native kubelet PodResources client (csrc/core/grpc_lite.cpp: HTTP/2 + gRPC + protobuf by hand)
against the in-process fake kubelet (a real grpcio server on a unix socket), and the exporter's
native poller that turns allocations into idle pod_gpu rows for the standalone binary."""

import os
import subprocess
import time
import urllib.request

import pytest

from gpumon.attribution.fake_kubelet import FakeKubelet, FakePod
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
    from gpumon.attribution import proto as P

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
