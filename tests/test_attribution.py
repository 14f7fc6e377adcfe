"""PID -> container -> pod attribution and the reference's user-name / opt-in rules.

Reference behaviour being reproduced (or deliberately fixed):
  * gpu.py:196-199  user_name from pod name ("turing-gpu-notebook-<user>-<x>-<y>" or "<a>-<user>-...")
  * gpu.py:199      IndexError crash for pod names without '-'   (quirk Q2 -> "-")
  * gpu.py:184-188  opt-in label mlgpu == "mlgpu"
  * gpu.py:177      docker top pid list -> here /proc/<pid>/cgroup parsing (all runtimes / cgroup versions)
"""

import os

import pytest

CID = "3f2a" * 16  # 64 hex
UID = "1b4e28ba-2fa1-11d2-883f-0016d3cca427"


@pytest.mark.parametrize("text,runtime,cid,uid,qos", [
    # cgroup v1, cgroupfs driver, docker
    (f"12:memory:/kubepods/burstable/pod{UID}/{CID}\n11:cpu:/kubepods/burstable/pod{UID}/{CID}\n",
     "cgroupfs", CID, UID, "burstable"),
    # cgroup v1, systemd driver, docker
    (f"4:pids:/kubepods.slice/kubepods-besteffort.slice/kubepods-besteffort-pod{UID.replace('-', '_')}.slice/docker-{CID}.scope\n",
     "docker", CID, UID, "besteffort"),
    # cgroup v2, containerd, guaranteed QoS
    (f"0::/kubepods.slice/kubepods-pod{UID.replace('-', '_')}.slice/cri-containerd-{CID}.scope\n",
     "containerd", CID, UID, "guaranteed"),
    # cri-o
    (f"0::/kubepods.slice/kubepods-burstable.slice/kubepods-burstable-pod{UID.replace('-', '_')}.slice/crio-{CID}.scope\n",
     "crio", CID, UID, "burstable"),
    # plain docker (no k8s)
    (f"0::/system.slice/docker-{CID}.scope\n", "docker", CID, "", ""),
    (f"13:name=systemd:/docker/{CID}\n", "docker", CID, "", ""),
    # podman (rootful, systemd cgroup manager)
    (f"0::/machine.slice/libpod-{CID}.scope/container\n", "podman", CID, "", ""),
])
def test_parse_cgroup_formats(core, text, runtime, cid, uid, qos):
    r = core.parse_cgroup(text)
    assert r["found"]
    assert r["runtime"] == runtime
    assert r["container_id"] == cid
    assert r["pod_uid"] == uid
    assert r["qos"] == qos


# What /proc/<pid>/cgroup says on a real container runtime (gpurun call r4a, tools/runtime_cgroup_probe.py,
# profiles/r4_runtime_attribution.md; the 32-hex id replaced): a cgroup v2 host whose runtime puts each
# container in /<manager>/<32-hex id> -- the exporter, and a torch tenant holding /dev/kfd, share it;
# the box's init sits in /<manager>/core. And what a DaemonSet pod with a private cgroup namespace
# reads for another pod's process: a path relative to its own namespace root ("/../..").
BOX_ID = "5e1f" * 8


@pytest.mark.parametrize("text,found,runtime,cid,uid,qos", [
    (f"0::/process_api/{BOX_ID}\n", True, "cgroupfs", BOX_ID, "", ""),
    ("0::/process_api/core\n", False, "", "", "", ""),
    (f"0::/../../kubepods-besteffort-pod{UID.replace('-', '_')}.slice/cri-containerd-{CID}.scope\n",
     True, "containerd", CID, UID, "besteffort"),
    (f"0::/../kubepods/burstable/pod{UID}/{CID}\n", True, "cgroupfs", CID, UID, "burstable"),
])
def test_parse_cgroup_observed_and_namespaced(core, text, found, runtime, cid, uid, qos):
    r = core.parse_cgroup(text)
    assert (r["found"], r["runtime"], r["container_id"], r["pod_uid"], r["qos"]) == (found, runtime, cid, uid, qos)


def test_parse_cgroup_host_process(core):
    r = core.parse_cgroup("0::/user.slice/user-1000.slice/session-3.scope\n")
    assert not r["found"] and r["container_id"] == ""


def test_parse_cgroup_ignores_crio_conmon(core):
    r = core.parse_cgroup(f"0::/kubepods.slice/crio-conmon-{CID}.scope\n")
    assert not r["found"]


@pytest.mark.parametrize("pod,user", [
    ("turing-gpu-notebook-alice-7d9f8-x2x", "alice"),        # rsplit("-", 2)[0]
    ("turing-gpu-notebook-bob-smith-5c7-abc", "bob-smith"),
    ("turing-gpu-notebook-carol", "carol"),
    ("jupyter-w-0", "w"),                                     # split("-")[1]  (2019 screenshot: users e/q/w)
    ("train-dave-job-5", "dave"),
    ("nodash", "-"),                                          # reference crashes here (Q2)
    ("", "-"),
    ("-", "-"),
])
def test_compat_user_rule(core, pod, user):
    assert core.compat_user_from_pod(pod) == user


def _reference_user(podname):
    """Literal transcription of gpu.py:196-199 (for cross-checking the C++ rule)."""
    if "turing-gpu-notebook-" in podname:
        return podname.split("turing-gpu-notebook-")[1].rsplit("-", 2)[0]
    return podname.split("-")[1]


@pytest.mark.parametrize("pod", ["turing-gpu-notebook-x-y-z", "a-b", "a-b-c-d", "turing-gpu-notebook-u-v",
                                 "x-turing-gpu-notebook-eve-1-2", "m--n"])
def test_compat_rule_equals_reference_where_reference_does_not_crash(core, pod):
    ref = _reference_user(pod)
    assert core.compat_user_from_pod(pod) == (ref if ref else "-")


def test_user_regex_and_label_override(mock_exporter):
    ex = mock_exporter(user_regex=r"^nb-([a-z]+)-", user_label="example.com/user")
    assert ex.derive_user("nb-zoe-0", {}) == "zoe"
    assert ex.derive_user("nb-zoe-0", {"example.com/user": "zed"}) == "zed"
    assert ex.derive_user("other-pod-1", {}) == "pod"  # falls back to the compat rule


def _fake_proc(tmp_path, pid, cgroup, comm="python3", env=None, ns=None):
    d = tmp_path / str(pid)
    d.mkdir(parents=True)
    (d / "stat").write_text(f"{pid} ({comm}) S 1 1 1 0 -1 4194560 100 0 0 0 5 3 0 0 20 0 8 0 424242 1000 100\n")
    (d / "cgroup").write_text(cgroup)
    if env:
        (d / "environ").write_bytes(b"\0".join(f"{k}={v}".encode() for k, v in env.items()) + b"\0")
    if ns:
        sa = d / "root/var/run/secrets/kubernetes.io/serviceaccount"
        sa.mkdir(parents=True)
        (sa / "namespace").write_text(ns)


def test_resolve_pid_via_meta_table(mock_exporter, tmp_path):
    _fake_proc(tmp_path, 4242, f"0::/kubepods.slice/kubepods-pod{UID.replace('-', '_')}.slice/cri-containerd-{CID}.scope\n")
    ex = mock_exporter(procfs_root=str(tmp_path))
    ex.set_container_meta([{"container_id": CID, "container_name": "main", "pod_name": "turing-gpu-notebook-alice-5f-x",
                            "pod_namespace": "ml", "pod_uid": UID, "labels": {"mlgpu": "mlgpu"}}])
    r = ex.resolve_pid(4242)
    assert r["valid"] and r["in_container"] and r["source"] == "meta"
    assert (r["pod_name"], r["pod_namespace"], r["container_name"], r["user_name"]) == (
        "turing-gpu-notebook-alice-5f-x", "ml", "main", "alice")
    assert r["comm"] == "python3"


def test_resolve_pid_procfs_fallback(mock_exporter, tmp_path):
    _fake_proc(tmp_path, 77, f"0::/kubepods.slice/cri-containerd-{CID}.scope\n",
               env={"HOSTNAME": "jupyter-q-0", "PATH": "/bin"}, ns="research")
    ex = mock_exporter(procfs_root=str(tmp_path))
    r = ex.resolve_pid(77)
    assert r["source"] == "procfs"
    assert (r["pod_name"], r["pod_namespace"], r["user_name"]) == ("jupyter-q-0", "research", "q")


def test_resolve_unknown_pid(mock_exporter, tmp_path):
    ex = mock_exporter(procfs_root=str(tmp_path))
    assert not ex.resolve_pid(999999)["valid"]


def test_opt_in_gate_filters_pod_rows(mock_exporter, tmp_path):
    cid2 = "ab" * 32
    _fake_proc(tmp_path, 100, f"0::/kubepods.slice/cri-containerd-{CID}.scope\n")
    _fake_proc(tmp_path, 101, f"0::/kubepods.slice/cri-containerd-{cid2}.scope\n")
    ex = mock_exporter(backend="mock:gpus=2", procfs_root=str(tmp_path), opt_in="mlgpu=mlgpu")
    ex.set_container_meta([
        {"container_id": CID, "container_name": "c", "pod_name": "jupyter-e-0", "pod_namespace": "ml",
         "labels": {"mlgpu": "mlgpu"}},
        {"container_id": cid2, "container_name": "c", "pod_name": "jupyter-w-0", "pod_namespace": "ml",
         "labels": {}},
    ])
    ex.mock_set_procs([{"pid": 100, "device": 0, "vram_bytes": 3 << 30}, {"pid": 101, "device": 1}])
    ex.tick()
    rows = ex.pod_rows()
    assert [(r["pid"], r["podname"], r["user_name"], r["containerid"]) for r in rows] == [
        ("100", "jupyter-e-0", "e", CID[:12])]
    assert rows[0]["used_memory_bytes"] == 3 << 30


def test_idle_allocation_rows(mock_exporter, tmp_path):
    """Reference gpu.py:220-253: an opted-in container holding a GPU with no process gets a row
    with pid "-", procressname "-", gpu_util 0, used_memory 0."""
    from gpumon.export import promtext

    ex = mock_exporter(backend="mock:gpus=2", procfs_root=str(tmp_path))
    ex.set_allocations([
        {"pod_namespace": "ml", "pod_name": "turing-gpu-notebook-bob-1-2", "container_name": "nb",
         "container_id": CID, "gpu_index": 1, "labels": {}},
        {"pod_namespace": "ml", "pod_name": "ghost", "container_name": "x", "gpu_index": 7},  # unknown GPU: skipped (Q5)
    ])
    ex.tick()
    rows = ex.pod_rows()
    assert len(rows) == 1
    r = rows[0]
    assert (r["idle"], r["pid"], r["procname"], r["user_name"], r["gpu_util"], r["used_memory_bytes"]) == (
        True, "-", "-", "bob", 0, 0)
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "pod_gpu_used_memory", pid="-", gpu_id="1") == 0
    assert promtext.one(fam, "pod_gpu_allocated", podname="turing-gpu-notebook-bob-1-2", state="idle") == 1
    assert promtext.one(fam, "gpumon_gpus", state="allocated_idle") == 1
    assert promtext.one(fam, "gpumon_gpus", state="allocated_active") == 0
    lines = [l for l in ex.influx_text().splitlines() if l.startswith("pod_gpu,")]
    assert len(lines) == 1 and "pid_t=-" in lines[0] and "gpu_util=0,used_memory=0" in lines[0]


def test_active_process_suppresses_idle_row(mock_exporter, tmp_path):
    _fake_proc(tmp_path, 555, f"0::/kubepods.slice/cri-containerd-{CID}.scope\n")
    ex = mock_exporter(backend="mock:gpus=1", procfs_root=str(tmp_path))
    ex.set_container_meta([{"container_id": CID, "container_name": "nb", "pod_name": "jupyter-q-0",
                            "pod_namespace": "ml"}])
    ex.set_allocations([{"pod_namespace": "ml", "pod_name": "jupyter-q-0", "container_name": "nb",
                         "container_id": CID, "gpu_index": 0}])
    ex.mock_set_procs([{"pid": 555, "device": 0}])
    ex.tick()
    rows = ex.pod_rows()
    assert len(rows) == 1 and not rows[0]["idle"]


def test_host_processes_toggle(mock_exporter, tmp_path):
    _fake_proc(tmp_path, 9, "0::/user.slice/session-1.scope\n")
    ex = mock_exporter(procfs_root=str(tmp_path), include_host_processes=False)
    ex.mock_set_procs([{"pid": 9, "device": 0}])
    ex.tick()
    assert ex.pod_rows() == []


def test_bare_metal_host_process_is_a_row_with_dash_labels(mock_exporter, tmp_path):
    """deploy/systemd/ (no kubelet): a GPU process in a login session or a Slurm job step is a row
    with its pid and process name; the pod, namespace and container labels read "-"."""
    _fake_proc(tmp_path, 9, "0::/user.slice/session-1.scope\n", comm="train.py")
    _fake_proc(tmp_path, 10, "0::/system.slice/slurmstepd.scope/job_42/step_0/user/task_0\n", comm="python3")
    ex = mock_exporter(procfs_root=str(tmp_path), include_host_processes=True)
    ex.mock_set_procs([{"pid": 9, "device": 0, "vram_bytes": 1 << 30}, {"pid": 10, "device": 1, "vram_bytes": 1 << 30}])
    ex.tick()
    rows = sorted(ex.pod_rows(), key=lambda r: r["pid"])
    assert [(r["pid"], r["dev"]) for r in rows] == [("10", 1), ("9", 0)]
    for r in rows:
        assert r["podname"] == "-" and r["namespace"] == "-" and r["container"] == "-" and not r["idle"]


def test_proc_gfx_util_from_engine_ns(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=1,mode=load")
    ex.mock_set_procs([{"pid": os.getpid(), "device": 0, "gfx_share": 0.5}])
    ex.tick()
    import time

    time.sleep(0.05)
    ex.tick()
    r = ex.pod_rows()[0]
    assert r["proc_gfx_util"] is not None and 0 < r["proc_gfx_util"] <= 100


def test_kfd_handle_check_rejects_foreign_pid(core, tmp_path):
    """amdsmi PIDs are host-namespace PIDs; a same-numbered process in our /proc that does not
    hold /dev/kfd must not be attributed (exporter running without hostPID)."""
    _fake_proc(tmp_path, 300, f"0::/kubepods.slice/cri-containerd-{CID}.scope\n")
    (tmp_path / "300" / "fd").mkdir()
    os.symlink("/dev/null", tmp_path / "300" / "fd" / "0")
    _fake_proc(tmp_path, 301, f"0::/kubepods.slice/cri-containerd-{CID}.scope\n")
    (tmp_path / "301" / "fd").mkdir()
    os.symlink("/dev/null", tmp_path / "301" / "fd" / "0")
    os.symlink("/dev/kfd", tmp_path / "301" / "fd" / "5")
    ex = core.Exporter({"backend": "amdsmi", "serve_http": False, "interval_s": 0, "procfs_root": str(tmp_path)})
    r300, r301 = ex.resolve_pid(300), ex.resolve_pid(301)
    assert r300["pid_mismatch"] and not r300["valid"] and r300["container_id"] == ""
    assert r301["valid"] and not r301["pid_mismatch"] and r301["container_id"] == CID


@pytest.mark.parametrize("comm,tail,start", [
    ("python3", "S 1 1 1 0 -1 4194560 100 0 0 0 5 3 0 0 20 0 8 0 424242 1000 100", 424242),
    ("a) b (c", "S 1 1 1 0 -1 4194560 100 0 0 0 5 3 0 0 20 0 8 0 777 1000 100", 777),  # parens in comm
    ("x y", "S 1 1 1 0 -1 4194560 100 0 0 0 5 3 0 0 20 0 8 0 31337", 31337),  # starttime is the last field
    ("short", "S 1 1 1", 0),  # truncated stat: no starttime
])
def test_stat_starttime_and_comm(mock_exporter, tmp_path, comm, tail, start):
    """/proc/<pid>/stat: comm is the text between the first '(' and the LAST ')', starttime is the
    22nd field (the pid-reuse key of the attribution cache)."""
    d = tmp_path / "55"
    d.mkdir()
    (d / "stat").write_text(f"55 ({comm}) {tail}\n")
    (d / "cgroup").write_text("0::/\n")
    ex = mock_exporter(procfs_root=str(tmp_path))
    r = ex.resolve_pid(55)
    assert r["comm"] == comm or not r["valid"]
    assert r["starttime"] == start
