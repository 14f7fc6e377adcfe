"""The canonical 8-GPU tenant: one pod running 8 torchrun ranks, one rank per GPU.

Each rank's runtime opens every GPU of the node. It holds a KFD context, and with RCCL's imported
peer buffers some VRAM, on all 8. It runs waves only on its own GPU. The reference emitted one
pod_gpu row per compute app that nvidia-smi listed on a GPU (/root/reference/gpu.py:111-116,178,
190-219). A rank shows up there on its own GPU. Its "GPUs held per user" panel is `pod_gpu.count`
grouped by user_name_t. For this pod it must read 8, not 64.

The rule (csrc/core/pod_rows.cpp build_pod_rows) calls a (pid, GPU) context a peer context when,
on that GPU, it:
* holds at most `peer_context_max_vram_mib`;
* had no resident wave within the sharing window, where occupancy is readable;
* belongs to a process with a workload context on another GPU.

A peer context gets no pod_gpu row and is not a sharer in gpu_active_processes. It is counted in
gpumon_hidden_peer_gpu_contexts. A process that uses only small amounts of VRAM, and only on one GPU,
keeps its row.
"""

import collections

import pytest

from gpumon.export import promtext

CID = "0123456789ab" * 5 + "cdef"
UID = "5b0c1d2e-0000-4000-8000-00000000abcd"


def _fake_proc(tmp_path, pid, cgroup, comm="python3"):
    d = tmp_path / str(pid)
    d.mkdir(parents=True)
    (d / "stat").write_text(f"{pid} ({comm}) S 1 1 1 0 -1 4194560 100 0 0 0 5 3 0 0 20 0 8 0 424242 1000 100\n")
    (d / "cgroup").write_text(cgroup)


def _ranks(peer_vram_mib=96, own_vram_gib=40, peer_gpus=range(8), queues=False):
    """`queues`: KFD's per-process queue list is readable (the sysfs fast path): each rank holds
    2 queues on its own GPU and none on the peers (measured on MI355X, profiles/r6_kfd_queues.md)."""
    procs = []
    for r in range(8):
        for g in peer_gpus:
            own = g == r
            p = {"pid": 1000 + r, "device": g, "name": "python3", "kfd_only": True,
                 "vram_bytes": (own_vram_gib << 30) if own else peer_vram_mib << 20,
                 "gfx_share": 1.0 if own else 0.0}
            if queues:
                p["queues"] = 2 if own else 0
            procs.append(p)
    return procs


@pytest.fixture
def torchrun_pod(mock_exporter, tmp_path):
    """8 ranks in one container of pod turing-gpu-notebook-alice-0 (user alice)."""
    for r in range(8):
        _fake_proc(tmp_path, 1000 + r,
                   f"0::/kubepods.slice/kubepods-pod{UID.replace('-', '_')}.slice/cri-containerd-{CID}.scope\n")

    def make(procs, **over):
        ex = mock_exporter(backend="mock:gpus=8,mode=const,const_util=95", sample_threads=0, procfs_root=str(tmp_path),
                           mock={"procs": procs}, **over)
        ex.set_container_meta([{"container_id": CID, "container_name": "trainer", "pod_name": "turing-gpu-notebook-alice-0",
                                "pod_namespace": "ml", "pod_uid": UID, "labels": {}}])
        ex.set_allocations([{"pod_namespace": "ml", "pod_name": "turing-gpu-notebook-alice-0", "container_name": "trainer",
                             "container_id": CID, "gpu_index": g, "labels": {}} for g in range(8)])
        for _ in range(3):
            ex.tick()
        return ex

    return make


def _workload_rows(ex):
    return [r for r in ex.pod_rows() if not r["idle"]]


@pytest.mark.parametrize("peer_vram_mib", [0, 4, 96, 384])
def test_every_rank_on_every_gpu_gives_one_row_per_gpu(torchrun_pod, peer_vram_mib):
    ex = torchrun_pod(_ranks(peer_vram_mib=peer_vram_mib))
    rows = _workload_rows(ex)
    per_gpu = collections.Counter(r["dev"] for r in rows)
    assert per_gpu == {g: 1 for g in range(8)}, per_gpu
    assert {(r["dev"], r["pid"]) for r in rows} == {(g, str(1000 + g)) for g in range(8)}
    assert all(r["used_memory_bytes"] == 40 << 30 for r in rows)
    # the reference's "GPUs held per user" panel: pod_gpu.count by user_name_t
    assert collections.Counter(r["user_name"] for r in rows) == {"alice": 8}
    # no idle-allocation row: every allocated GPU has its rank's row
    assert not [r for r in ex.pod_rows() if r["idle"]]
    st = ex.self_stats()
    hidden = 56 if peer_vram_mib else 0
    assert st["hidden_peer_contexts"] == hidden
    assert st["hidden_contexts"] == (0 if peer_vram_mib else 56)  # no VRAM at all: the empty-context rule
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpumon_hidden_peer_gpu_contexts") == hidden
    # every GPU is exclusive to its rank: 1 active process each, not 8
    assert sorted(v for _, _, v in fam["gpu_active_processes"]["samples"]) == [1.0] * 8
    assert promtext.one(fam, "gpumon_gpus", state="allocated_active") == 8
    assert len(fam["pod_gpu_used_memory"]["samples"]) == 8
    # the Influx compat push: 8 pod_gpu lines (reference: one per listed compute app)
    assert sum(l.startswith("pod_gpu,") for l in ex.influx_text().splitlines()) == 8


def test_peer_context_with_much_vram_is_a_workload(torchrun_pod):
    """Above peer_context_max_vram_mib a context is a workload even without waves (model shards held
    on a GPU that is idle this window): rows on every GPU, as the reference would list them."""
    ex = torchrun_pod(_ranks(peer_vram_mib=2048))
    assert len(_workload_rows(ex)) == 64
    assert ex.self_stats()["hidden_peer_contexts"] == 0


def test_rule_off_restores_the_raw_contexts(torchrun_pod):
    ex = torchrun_pod(_ranks(peer_vram_mib=96), peer_context_max_vram_mib=0.0)
    assert len(_workload_rows(ex)) == 64
    # 0 turns the queue rule off too: every context with VRAM is a row again
    ex = torchrun_pod(_ranks(peer_vram_mib=96, queues=True), peer_context_max_vram_mib=0.0)
    assert len(_workload_rows(ex)) == 64 and ex.self_stats()["hidden_peer_contexts"] == 0


def test_small_single_gpu_process_keeps_its_row(mock_exporter):
    """Only a process with real work on ANOTHER GPU loses a small idle context: a notebook holding
    64 MiB on one GPU with no waves is still a row."""
    ex = mock_exporter(backend="mock:gpus=2,mode=const,const_util=50", sample_threads=0,
                       mock={"procs": [{"pid": 77, "device": 1, "kfd_only": True, "vram_bytes": 64 << 20,
                                        "gfx_share": 0.0}]})
    for _ in range(2):
        ex.tick()
    assert [(r["dev"], r["pid"]) for r in _workload_rows(ex)] == [(1, "77")]
    assert ex.self_stats()["hidden_peer_contexts"] == 0


def test_waves_on_a_peer_gpu_make_it_a_workload(torchrun_pod):
    """A rank that really computes on a second GPU (waves there) keeps that row too."""
    procs = _ranks(peer_vram_mib=96)
    for p in procs:
        if p["pid"] == 1000 and p["device"] == 1:
            p["gfx_share"] = 0.5
    ex = torchrun_pod(procs)
    rows = _workload_rows(ex)
    assert collections.Counter(r["dev"] for r in rows)[1] == 2
    assert {r["pid"] for r in rows if r["dev"] == 1} == {"1000", "1001"}



# ---------------------------------------------------------------- KFD queues
@pytest.mark.parametrize("peer_vram_mib", [96, 2048, 16384])
def test_queue_list_hides_peer_contexts_whatever_their_vram(torchrun_pod, peer_vram_mib):
    """Where KFD lists each process's hardware queues, a context with no queue on its GPU and no
    waves there is a peer context however much VRAM it holds: 8 rows for 8 ranks, also when the
    threshold rule alone would have made 64 (test_peer_context_with_much_vram_is_a_workload)."""
    ex = torchrun_pod(_ranks(peer_vram_mib=peer_vram_mib, queues=True))
    rows = _workload_rows(ex)
    assert {(r["dev"], r["pid"]) for r in rows} == {(g, str(1000 + g)) for g in range(8)}
    assert ex.self_stats()["hidden_peer_contexts"] == 56
    # /debug/procs names each of the 56 with the reason: rank g's context on every other GPU
    hidden = [(c["dev"], c["pid"]) for c in ex.debug_view("/debug/procs") if c["why"] == "peer"]
    assert sorted(hidden) == sorted((d, 1000 + g) for g in range(8) for d in range(8) if d != g)


def _tp_pair(queues):
    """A tensor / pipeline-parallel process (pid 2000): its main shard on GPU 0 with waves, a 100 MiB
    shard on GPU 1 that it also computes on (queues there) but had no wave resident in the window."""
    q0, q1 = (2, 2) if queues else (-1, -1)
    return [{"pid": 2000, "device": 0, "kfd_only": True, "vram_bytes": 30 << 30, "gfx_share": 1.0, "queues": q0},
            {"pid": 2000, "device": 1, "kfd_only": True, "vram_bytes": 100 << 20, "gfx_share": 0.0, "queues": q1}]


def test_tp_process_with_a_small_idle_shard_keeps_its_row(mock_exporter):
    """VERDICT r5 #3 done-means: a TP / PP process with a < 512 MiB idle shard keeps that row when
    KFD shows it holds queues on that GPU (the VRAM threshold alone hid it: next test)."""
    ex = mock_exporter(backend="mock:gpus=2,mode=const,const_util=50", sample_threads=0,
                       mock={"procs": _tp_pair(queues=True)})
    for _ in range(3):
        ex.tick()
    assert sorted((r["dev"], r["pid"]) for r in _workload_rows(ex)) == [(0, "2000"), (1, "2000")]
    assert ex.self_stats()["hidden_peer_contexts"] == 0


def test_without_a_queue_list_the_vram_threshold_still_applies(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=2,mode=const,const_util=50", sample_threads=0,
                       mock={"procs": _tp_pair(queues=False)})
    for _ in range(3):
        ex.tick()
    assert [(r["dev"], r["pid"]) for r in _workload_rows(ex)] == [(0, "2000")]
    assert ex.self_stats()["hidden_peer_contexts"] == 1


def test_allocate_only_single_gpu_process_keeps_its_row(mock_exporter):
    """No queue anywhere and no other GPU: not a peer context (a job still starting up, a notebook
    that only allocated) -- the rule needs a workload on another GPU."""
    ex = mock_exporter(backend="mock:gpus=2,mode=const,const_util=50", sample_threads=0,
                       mock={"procs": [{"pid": 88, "device": 1, "kfd_only": True, "vram_bytes": 1 << 30,
                                        "gfx_share": 0.0, "queues": 0}]})
    for _ in range(2):
        ex.tick()
    assert [(r["dev"], r["pid"]) for r in _workload_rows(ex)] == [(1, "88")]
