"""Multi-GPU hardware validation of the xGMI fields: skipped on a box with fewer
than 2 GPUs, run by the GPU tier on a full node. The reference is one agent per node covering
every GPU (/root/reference/gpu_monitor.yaml:1-5,19-20; the per-GPU loop at gpu.py:132).

(a) link map: GPU i pushes into GPU j (native XgmiLoad); the link whose write counter moves on i
    must be the one the exporter maps to j's BDF, and its rate must match the copy's own rate;
(b) single-process bench over every GPU: each GPU loaded, the peer-copy ring's traffic seen per GPU;
(c) torchrun bench: RCCL ring all-reduce traffic per GPU = 2(N-1)/N x bytes / t.
"""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpus():
    """GPUs in the KFD topology (gpu_id != 0). Counted WITHOUT touching HIP: initialising a HIP
    runtime at collection time, before torch brings up its own, leaves torch without a GPU."""
    import glob

    n = 0
    for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            n += int(open(p).read().strip() or 0) != 0
        except (OSError, ValueError):
            pass
    return n


N = _gpus()
needs2 = pytest.mark.skipif(N < 2, reason=f"needs >= 2 GPUs (found {N})")


@needs2
def test_every_peer_link_maps_to_its_bdf_and_rate():
    from gpumon import core
    from gpumon.parallel.devmap import hip_bdfs, index_of, match
    from gpumon.parallel.xgmi import rate_within, validate_pair

    n = min(N, 8)
    bdfs = hip_bdfs(range(n))  # HIP ordinal -> PCI address: the exporter samples exactly these
    ex = core().Exporter({"backend": "amdsmi", "devices": [bdfs[k] for k in range(n)], "serve_http": False,
                          "interval_s": 0.1, "link_every": 1, "processes": False})
    assert ex.start() == ""
    bad = []
    try:
        idx = index_of(match(bdfs, ex.statics()))
        for src in range(n):
            for dst in range(n):
                if src == dst:
                    continue
                r = validate_pair(ex, src, dst, seconds=0.6, interval=0.1, index_of=idx)
                if not (r["peer_matches"] and rate_within(r, 0.15)):
                    bad.append(r)
    finally:
        ex.stop()
    assert not bad, json.dumps(bad[:4], indent=1)


def _bench(cmd, timeout):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


@needs2
def test_single_process_bench_loads_every_gpu_and_sees_the_copy_ring():
    n = min(N, 8)
    d = _bench([sys.executable, "bench.py", "--gpus", str(n), "--steps", "5", "--warmup", "2",
                "--interval", "0.5", "--link-check-s", "0"], 400)
    assert d["sampled_devices"] == n and d["scrape_errors"] == 0
    assert sorted(r["hip_ordinal"] for r in d["devices"]) == list(range(n)) and d["device_check"]["ok"], d["devices"]
    assert all(g["tflops"] > 500 for g in d["load_per_gpu"]), d["load_per_gpu"]
    x = d["xgmi"]
    assert x["mode"] == "peer_copy_ring"
    for g in x["per_gpu"]:
        # the copy kernel STORES into the peer: the source's write counter carries it (whether the
        # receiver's read counter also counts incoming writes is reported, not asserted)
        assert abs(g["tx_vs_expected"] - 1) <= 0.15, g


@needs2
def test_torchrun_allreduce_traffic_per_gpu_matches_the_ring():
    n = min(N, 8)
    d = _bench([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 400), "bench.py",
                "--gpus", str(n), "--steps", "6", "--warmup", "2", "--interval", "0.5"], 600)
    x = d["xgmi"]
    assert x["mode"] == "rccl_allreduce" and x["allreduces_per_step"] >= 1
    for g in x["per_gpu"]:
        # a ring moves the same bytes out of and into every GPU; RCCL's P2P transport may push
        # (writes) or pull (reads), so the traffic shows in one direction's counter or both
        best = max(g.get("tx_vs_expected") or 0, g.get("rx_vs_expected") or 0)
        assert abs(best - 1) <= 0.15, g
    lm = x["link_map"]
    assert lm["peers_matched"] == lm["peers"] == n - 1, lm
