"""Socket-free pod metadata for a non-root exporter (csrc/core/kubelet_files.cpp):
container id -> pod / namespace / container from the kubelet's /var/log/containers symlink names,
pod uid from /var/log/pods, and GPU allocations (idle rows) from the device-plugin checkpoint.
The reference needed the root-equivalent docker.sock for the same data
(/root/reference/gpu.py:86-103,177; gpu_monitor.yaml:24-28)."""

import json
import os

import pytest

from gpumon.export import promtext

CID_A = "a" * 63 + "1"
CID_B = "b" * 63 + "2"
UID_A = "1f0c6a8e-5d1b-4c53-9f8e-0000000000a1"
UID_B = "2e1d7b9f-6e2c-4d64-8a9f-0000000000b2"


def _fake_proc(root, pid, cgroup_line):
    d = root / str(pid)
    d.mkdir(parents=True)
    (d / "stat").write_text(f"{pid} (python) S 1 1 1 0 -1 0 0 0 0 0 0 0 0 0 20 0 1 0 777 0 0\n")
    (d / "cgroup").write_text(cgroup_line + "\n")


def _log_tree(root):
    pods, ctrs = root / "pods", root / "containers"
    for ns, pod, uid, ctr, cid in (("ml", "turing-gpu-notebook-alice-5d8f-x1", UID_A, "notebook", CID_A),
                                   ("research", "jupyter-q-0", UID_B, "main", CID_B)):
        (pods / f"{ns}_{pod}_{uid}" / ctr).mkdir(parents=True)
        ctrs.mkdir(exist_ok=True)
        os.symlink(f"/var/log/pods/{ns}_{pod}_{uid}/{ctr}/0.log", ctrs / f"{pod}_{ns}_{ctr}-{cid}.log")
    (ctrs / "not-a-kubelet-log.txt").write_text("")  # ignored


def _checkpoint(path, v1=False):
    def ids(x):
        return x if v1 else {"0": x}

    entries = [
        {"PodUID": UID_A, "ContainerName": "notebook", "ResourceName": "amd.com/gpu",
         "DeviceIDs": ids(["0000:05:00.0"]), "AllocResp": "Cg=="},
        {"PodUID": UID_B, "ContainerName": "main", "ResourceName": "amd.com/gpu",
         "DeviceIDs": ids(["0000:25:00.0"]), "AllocResp": "Cg=="},
        {"PodUID": UID_B, "ContainerName": "main", "ResourceName": "example.com/nic",
         "DeviceIDs": ids(["eth9"]), "AllocResp": ""},
        {"PodUID": "gone-pod-uid", "ContainerName": "c", "ResourceName": "amd.com/gpu",
         "DeviceIDs": ids(["0000:45:00.0"]), "AllocResp": ""},  # pod no longer on the node
    ]
    body = {"Data": {"PodDeviceEntries": entries, "RegisteredDevices": {"amd.com/gpu": ["0000:05:00.0"]}},
            "Checksum": 1234567}
    path.write_text(json.dumps(body))


def test_pod_metadata_and_idle_rows_without_any_socket(core, tmp_path):
    proc = tmp_path / "proc"
    _fake_proc(proc, 2000, f"0::/kubepods.slice/kubepods-pod{UID_A.replace('-', '_')}.slice/"
                           f"cri-containerd-{CID_A}.scope")
    # jupyter-q-0 is running (a process in its container), just not on a GPU
    _fake_proc(proc, 2001, f"0::/kubepods.slice/kubepods-pod{UID_B.replace('-', '_')}.slice/"
                           f"cri-containerd-{CID_B}.scope")
    logs = tmp_path / "log"
    _log_tree(logs)
    ckpt = tmp_path / "kubelet_internal_checkpoint"
    _checkpoint(ckpt)
    ex = core.Exporter({"backend": "mock:gpus=3", "serve_http": False, "interval_s": 0, "host": "n1",
                        "procfs_root": str(proc), "pod_log_root": str(logs), "device_checkpoint": str(ckpt)})
    assert ex.start() == ""
    try:
        ex.mock_set_procs([{"pid": 2000, "device": 0, "name": "python train.py", "vram_bytes": 5 << 30}])
        ex.tick()
        rows = {(r["dev"], r["idle"]): r for r in ex.pod_rows()}
        busy = rows[(0, False)]
        assert (busy["namespace"], busy["podname"], busy["container"], busy["containerid"]) == \
            ("ml", "turing-gpu-notebook-alice-5d8f-x1", "notebook", CID_A[:12])
        assert busy["user_name"] == "alice"  # the reference's user rule on the pod name (gpu.py:196-199)
        idle = rows[(1, True)]  # jupyter-q-0 holds GPU 1 (0000:25:00.0) and runs nothing on it
        assert (idle["namespace"], idle["podname"], idle["container"], idle["containerid"]) == \
            ("research", "jupyter-q-0", "main", CID_B[:12])
        assert (0, True) not in rows  # the allocation of GPU 0 is in use: no idle row
        assert not [r for r in ex.pod_rows() if r["dev"] == 2]  # the departed pod's GPU
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpumon_kubelet_files_up", source="pod_logs") == 1
        assert promtext.one(fam, "gpumon_kubelet_files_up", source="device_checkpoint") == 1
        assert promtext.one(fam, "gpumon_kubelet_files_containers") == 2
    finally:
        ex.stop()


def test_checkpoint_entry_of_a_finished_pod_is_not_an_idle_row(core, tmp_path):
    """the checkpoint keeps a Completed pod's entry (and the log tree its directory) until
    the pod is deleted. Its container has no live process, so it is no idle allocation: dropped
    and counted. A running pod's idle allocation stays."""
    proc = tmp_path / "proc"
    _fake_proc(proc, 2000, f"0::/kubepods.slice/kubepods-pod{UID_A.replace('-', '_')}.slice/"
                           f"cri-containerd-{CID_A}.scope")  # notebook pod: running (no GPU process)
    logs = tmp_path / "log"
    _log_tree(logs)  # jupyter-q-0 (CID_B) has its log dir and symlink, but no process: it completed
    ckpt = tmp_path / "ckpt"
    _checkpoint(ckpt)
    ex = core.Exporter({"backend": "mock:gpus=3", "serve_http": False, "interval_s": 0, "host": "n1",
                        "procfs_root": str(proc), "pod_log_root": str(logs), "device_checkpoint": str(ckpt)})
    assert ex.start() == ""
    try:
        ex.tick()
        idle = sorted((r["dev"], r["podname"]) for r in ex.pod_rows() if r["idle"])
        assert idle == [(0, "turing-gpu-notebook-alice-5d8f-x1")]
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpumon_kubelet_files_exited_allocations") == 1
    finally:
        ex.stop()


@pytest.mark.parametrize("dead_link_first", [True, False])
@pytest.mark.parametrize("old_cid", ["c" * 63 + "9", "0" * 63 + "1", "e" * 63 + "7", "9" * 63 + "5"])
def test_restarted_container_keeps_its_allocation(core, tmp_path, dead_link_first, old_cid):
    """after a container restart the kubelet keeps the dead instance's log link next to
    the new one until garbage collection. Whichever readdir lists last, the allocation of the still
    running pod stays an idle row carrying the LIVE instance's id, and is not counted as exited.
    (readdir order is the filesystem's: several dead ids and both creation orders cover it.)"""
    proc = tmp_path / "proc"
    _fake_proc(proc, 2000, f"0::/kubepods.slice/kubepods-pod{UID_A.replace('-', '_')}.slice/"
                           f"cri-containerd-{CID_A}.scope")  # the new notebook instance: running
    _fake_proc(proc, 2001, f"0::/kubepods.slice/kubepods-pod{UID_B.replace('-', '_')}.slice/"
                           f"cri-containerd-{CID_B}.scope")
    logs = tmp_path / "log"
    pod, ns, uid = "turing-gpu-notebook-alice-5d8f-x1", "ml", UID_A

    def dead_link():  # the dead instance (restart count 0 -> 1): its log link is still there
        (logs / "containers").mkdir(parents=True, exist_ok=True)
        os.symlink(f"/var/log/pods/{ns}_{pod}_{uid}/notebook/0.log",
                   logs / "containers" / f"{pod}_{ns}_notebook-{old_cid}.log")

    # readdir order follows creation order on some filesystems: both orders are checked
    if dead_link_first:
        dead_link()
    _log_tree(logs)
    if not dead_link_first:
        dead_link()
    ckpt = tmp_path / "ckpt"
    _checkpoint(ckpt)
    ex = core.Exporter({"backend": "mock:gpus=3", "serve_http": False, "interval_s": 0, "host": "n1",
                        "procfs_root": str(proc), "pod_log_root": str(logs), "device_checkpoint": str(ckpt)})
    assert ex.start() == ""
    try:
        ex.tick()
        idle = {r["dev"]: r for r in ex.pod_rows() if r["idle"]}
        assert sorted(idle) == [0, 1]
        assert idle[0]["podname"] == pod and idle[0]["containerid"] == CID_A[:12]
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpumon_kubelet_files_exited_allocations") == 0
    finally:
        ex.stop()


def test_checkpoint_v1_list_form_and_unreadable_files(core, tmp_path):
    """Older kubelets checkpoint DeviceIDs as a plain list; an unreadable or malformed file reports
    gpumon_kubelet_files_up 0 and keeps the exporter running."""
    logs = tmp_path / "log"
    _log_tree(logs)
    ckpt = tmp_path / "ckpt"
    _checkpoint(ckpt, v1=True)
    ex = core.Exporter({"backend": "mock:gpus=2", "serve_http": False, "interval_s": 0, "host": "n1",
                        "procfs_root": str(tmp_path / "proc"), "pod_log_root": str(logs),
                        "device_checkpoint": str(ckpt)})
    assert ex.start() == ""
    try:
        ex.tick()
        idle = sorted((r["dev"], r["podname"]) for r in ex.pod_rows() if r["idle"])
        assert idle == [(0, "turing-gpu-notebook-alice-5d8f-x1"), (1, "jupyter-q-0")]
    finally:
        ex.stop()
    ckpt.write_text('{"Data": {"PodDeviceEntries": [{"PodUID": ')  # truncated
    ex = core.Exporter({"backend": "mock:gpus=2", "serve_http": False, "interval_s": 0, "host": "n1",
                        "pod_log_root": str(tmp_path / "nope"), "device_checkpoint": str(ckpt)})
    assert ex.start() == ""
    try:
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpumon_kubelet_files_up", source="pod_logs") == 0
        assert promtext.one(fam, "gpumon_kubelet_files_up", source="device_checkpoint") == 0
        assert not [r for r in ex.pod_rows() if r["idle"]]
    finally:
        ex.stop()


def test_cri_metadata_wins_over_the_log_tree(core, tmp_path):
    """The files are the lowest-priority source: a container the CRI runtime (or Docker) reports
    keeps that metadata (labels included); the log tree only fills containers nobody else named."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from oracles.attribution.fake_kubelet import FakeKubelet, FakePod

    proc = tmp_path / "proc"
    _fake_proc(proc, 2000, f"0::/kubepods.slice/cri-containerd-{CID_A}.scope")
    _fake_proc(proc, 3000, f"0::/kubepods.slice/cri-containerd-{CID_B}.scope")
    logs = tmp_path / "log"
    _log_tree(logs)
    with FakeKubelet(podres_socket=str(tmp_path / "pr.sock"), cri_socket=str(tmp_path / "cri.sock")) as k:
        k.pods = [FakePod("renamed-by-cri-0", "ml", UID_A, labels={"team": "x"},
                          containers={"notebook": (CID_A, ["0000:05:00.0"])})]
        ex = core.Exporter({"backend": "mock:gpus=2", "serve_http": False, "interval_s": 0, "host": "n1",
                            "procfs_root": str(proc), "pod_log_root": str(logs), "cri_socket": k.cri_socket,
                            "label_allowlist": ["team"]})
        assert ex.start() == ""
        try:
            ex.mock_set_procs([{"pid": 2000, "device": 0, "vram_bytes": 1 << 30},
                               {"pid": 3000, "device": 1, "vram_bytes": 1 << 30}])
            ex.tick()
            by_pid = {r["pid"]: r for r in ex.pod_rows() if not r["idle"]}
            assert by_pid["2000"]["podname"] == "renamed-by-cri-0"  # CRI
            assert by_pid["3000"]["podname"] == "jupyter-q-0"  # the log tree fills the gap
        finally:
            ex.stop()


# ------------------------------------------------------------------ parsers (hypothesis)
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

_text = st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=20)
_entry = st.fixed_dictionaries(
    {"PodUID": _text.filter(bool), "ContainerName": _text, "ResourceName": _text,
     "DeviceIDs": st.one_of(st.lists(_text, max_size=3), st.dictionaries(st.sampled_from(["-1", "0", "1"]),
                                                                         st.lists(_text, max_size=3), max_size=2)),
     "AllocResp": _text},
    optional={"Extra": st.one_of(st.integers(), st.none(), st.lists(st.integers(), max_size=2))})


@settings(max_examples=200, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(entries=st.lists(_entry, max_size=5), extra=st.dictionaries(st.sampled_from(["RegisteredDevices", "X"]),
                                                                    st.integers(), max_size=2))
def test_checkpoint_parser_matches_python_json(core, entries, extra):
    body = json.dumps({"Data": {"PodDeviceEntries": entries, **extra}, "Checksum": 12345})
    got = core.device_checkpoint_parse(body.encode())
    want = []
    for e in entries:
        ids = e["DeviceIDs"] if isinstance(e["DeviceIDs"], list) else [x for v in e["DeviceIDs"].values() for x in v]
        want.append({"pod_uid": e["PodUID"].encode(), "container": e["ContainerName"].encode(),
                     "resource": e["ResourceName"].encode(), "device_ids": [x.encode() for x in ids]})
    assert got == want


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(raw=st.binary(max_size=200))
def test_checkpoint_parser_rejects_garbage_without_crashing(core, raw):
    try:
        core.device_checkpoint_parse(raw)
    except ValueError:
        pass


def test_container_log_names(core):
    cid = "0123456789abcdef" * 4
    assert core.container_log_name(f"my-pod-7f9_team-a_my-ctr-2-{cid}.log") == ("my-pod-7f9", "team-a", "my-ctr-2", cid)
    assert core.container_log_name(f"p.0_ns_c-{cid}.log") == ("p.0", "ns", "c", cid)
    for bad in (f"p_ns_c-{cid}.txt", f"p_ns_c-{cid[:-1]}.log", f"p_ns_x_c-{cid}.log", f"_ns_c-{cid}.log",
                f"p__c-{cid}.log", f"p_ns_-{cid}.log", "p_ns_c.log", f"p_ns_c-{cid.upper()}.log"):
        assert core.container_log_name(bad) is None, bad
