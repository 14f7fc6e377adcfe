#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): p99 /metrics scrape latency + samples/sec/GPU at 1 Hz.

    python bench.py [--gpus N --steps K --warmup W]                       # 1 process, N GPUs
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W           # N GPUs, one rank each

What one "step" is: one sampling period of the exporter (default 1 Hz, the BASELINE interval).
Rank 0 runs the SHIPPED exporter -- ``bin/gpumon-exporter --config <file>``, the image's
ENTRYPOINT, with the DaemonSet ConfigMap's keys -- as its own child process, started before this
process's first HIP call (``--exporter child``, the default; gpumon/export/child.py). The bench
process is then a foreign tenant to it, as every workload is in a cluster, and the exporter's tick
log, exact per-scrape service times, pod rows and self stats are read from its loopback-only
``debug_listen`` server; its CPU and RSS from /proc/<pid>. ``--exporter inprocess`` runs the same
core through the Python bindings inside this process instead (A/B). The exporter samples
exactly the GPUs the job loads (each HIP
ordinal paired with the exporter device of the same PCI BDF, gpumon/parallel/devmap.py, printed as
``devices``; the run fails if a loaded GPU reads under 50 % gfx_util, ``device_check``) and a
client-side scraper that hits /metrics at --scrape-rate, while EVERY GPU runs a synthetic gfx950 HIP load (bf16 MFMA burn +
HBM stream, csrc/hip/kernels.hip) and, for N > 1, xGMI traffic:

* under torchrun (one rank per GPU) each rank loads its own GPU and all ranks run RCCL ring
  all-reduces each step, as many as fill --xgmi-duty of the interval (calibrated before the timed
  region): every GPU's links carry 2(N-1)/N x bytes per all-reduce;
* in one process (``--gpus N`` without torchrun) the process loads all N GPUs and runs a native
  peer-copy ring (GPU i pushes into GPU (i+1) mod N, ``_hip.XgmiLoad``): each GPU's tx equals its
  copy rate.

Before any synthetic load starts, rank 0 runs the same scrape load for --idle-s seconds (untimed):
``scrape_idle`` holds that idle reference (scrape p50 / p99, tick cost), so every run reports the
BASELINE's "idle and under load" pair at its GPU count.

The exporter's own per-GPU xGMI counters are compared with that expectation
(``xgmi.per_gpu[].tx_vs_expected``), and after the timed region rank 0 drives GPU 0 -> k for every
peer k and checks that the link whose counter moves is the one the exporter maps to k's BDF
(``xgmi.link_map``). W warmup ticks, then exactly K ticks are timed between barriers +
torch.cuda.synchronize(); the MAX elapsed over ranks is used. The timed region starts right after
a tick and each step's xGMI traffic runs inside its own interval, so K steps span K intervals at
every N.

Reported ``value`` = whole-node fresh device samples per second (K ticks x N GPUs / elapsed);
``vs_baseline`` = per-GPU rate / 0.077 samples/s/GPU, the reference's best observed rate
(one node_gpu line per 13-19 s). The scrape-latency half of the headline metric is
reported as ``scrape_p99_ms`` / ``scrape_p999_ms`` / ``scrape_p50_ms`` (client-side, keep-alive,
like a Prometheus server, 200 req/s so a 10-tick run holds >= 2000 scrapes) and
``server_scrape_p99_ms`` (the exporter's own service time of the same requests, exact). Tick quantiles are exact over the timed ticks (the exporter's tick log). Without a GPU
the exporter uses the mock backend and says so in ``data``.

For the multi-GPU record the line also carries: every rank's view of the process group
(``ranks``: rank, world size, backend, pid, device), the exporter's CPU per thread
(``exporter_thread_cpu_millicores``), each sampled device's call times per tick
(``per_device_tick_ms``), the workload rows per GPU (``per_gpu_rows``), and the GPU contexts left
out of them with the exporter's reason (``hidden_context_reasons``, ``hidden_context_detail``:
empty / peer / helper / not opted in). ``--ranks-per-gpu K`` rehearses the torchrun path on a box
with fewer GPUs (K ranks per GPU over gloo, no xGMI; ``data`` says REHEARSAL).
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_METRIC = "p99 /metrics scrape latency + samples/sec/GPU at 1 Hz, 8×MI355X node"
BASELINE_SAMPLES_PER_GPU = 0.077  # best observed reference rate (1 node_gpu line / 13 s)


def _pct(xs, q):
    if not xs:
        return float("nan")
    xs = sorted(xs)
    k = (len(xs) - 1) * q
    f, c = math.floor(k), math.ceil(k)
    return xs[f] if f == c else xs[f] + (xs[c] - xs[f]) * (k - f)


def _ci(xs, q, n_boot=200, seed=1):
    """95 % bootstrap interval of the q-quantile (ms): how much a p99 over this many samples can
    move from resampling alone."""
    import random

    if len(xs) < 20:
        return None
    rnd = random.Random(seed)
    est = sorted(_pct([rnd.choice(xs) for _ in xs], q) for _ in range(n_boot))
    return [round(est[int(0.025 * n_boot)] * 1e3, 4), round(est[int(0.975 * n_boot) - 1] * 1e3, 4)]


def _r(x, nd=3):
    return round(x, nd) if isinstance(x, float) and x == x else x


def _server_durations(ex, n0, want, wait_s=1.0):
    """The exporter's own service times of the scrapes since count n0. The server logs a scrape
    after its response is written, so the client can hold the last response a moment before the
    server has logged it: wait (bounded) until the server has as many as the client counted."""
    t_end = time.monotonic() + wait_s
    while ex.scrape_count() - n0 < want and time.monotonic() < t_end:
        time.sleep(0.002)
    return list(ex.scrape_durations_since(n0))


def _per_gpu_xgmi(tick_rates, rows, expected_tx, expected_rx):
    """Exporter-measured xGMI tx / rx per GPU (sum over links, mean over the timed ticks; the first
    tick's rate spans part of the warmup and is skipped) against the traffic the bench drove.
    ``rows`` pair each loaded HIP ordinal with its exporter device (gpumon/parallel/devmap.py); the
    expectations are indexed by ordinal, the exporter's rates by device index."""
    ticks = tick_rates[1:] if len(tick_rates) > 1 else tick_rates
    out = []
    for m in rows:
        d, i = m["hip_ordinal"], m["index"]
        tx = [t[i][0] for t in ticks if i < len(t) and t[i] is not None]
        rx = [t[i][1] for t in ticks if i < len(t) and t[i] is not None]
        row = {"gpu": d, "gpu_id": m["gpu_id"],
               "exporter_tx_GBps": _r(sum(tx) / len(tx) / 1e9) if tx else None,
               "exporter_rx_GBps": _r(sum(rx) / len(rx) / 1e9) if rx else None,
               "expected_tx_GBps": _r(expected_tx[d] / 1e9) if expected_tx else None,
               "expected_rx_GBps": _r(expected_rx[d] / 1e9) if expected_rx else None}
        if tx and expected_tx and expected_tx[d] > 0:
            row["tx_vs_expected"] = _r(sum(tx) / len(tx) / expected_tx[d])
        if rx and expected_rx and expected_rx[d] > 0:
            row["rx_vs_expected"] = _r(sum(rx) / len(rx) / expected_rx[d])
        out.append(row)
    return out


def _bounded(fn, timeout_s, *args):
    """Run a post-measurement extra (link map, capacity) on a daemon thread and give up after
    timeout_s: the JSON line is the measurement, and a stuck validation call must not keep it from
    being printed."""
    out = {}

    def run():
        try:
            out["r"] = fn(*args)
        except Exception as e:  # noqa: BLE001
            out["r"] = {"error": f"{type(e).__name__}: {e}"}

    t = threading.Thread(target=run, daemon=True, name=f"bench-{fn.__name__}")
    t.start()
    t.join(timeout_s)
    return out.get("r", {"error": f"timed out after {timeout_s:g} s"})


def _link_map_check(ord_bdfs, seconds):
    """HIP ordinal 0 pushes into every peer in turn while a fresh 10 Hz exporter watches: the link
    whose write counter moves must be the one the exporter attributes to that peer's BDF."""
    from gpumon import core as _core
    from gpumon.parallel.devmap import index_of, match
    from gpumon.parallel.xgmi import rate_within, validate_pair

    n = len(ord_bdfs)
    ex = _core().Exporter({"backend": "amdsmi", "devices": [ord_bdfs[k] for k in sorted(ord_bdfs)],
                           "serve_http": False, "interval_s": 0.1, "link_every": 1, "processes": False,
                           "log_level": "warn"})
    err = ex.start()
    if err:
        return {"error": err}
    rows = []
    try:
        idx = index_of(match(ord_bdfs, ex.statics()))
        for k in range(1, n):
            r = validate_pair(ex, 0, k, seconds=seconds, interval=0.1, index_of=idx)
            r["rate_within_15pct"] = rate_within(r, 0.15)
            rows.append(r)
    finally:
        ex.stop()
    return {"pairs": rows, "peers_matched": sum(1 for r in rows if r["peer_matches"]), "peers": len(rows),
            "rates_within_15pct": sum(1 for r in rows if r["rate_within_15pct"])}


def _capacity(backend, devices, args, has_gpu):
    """Sampler capacity (untimed, after the timed region, load still running): a second exporter on
    the same devices at --capacity-interval (1 ms) for --capacity-s seconds. `value` is fixed by the
    configured interval; this is how fast the sampler can go: ticks/s, samples/s/GPU, the share of
    them that carried a new firmware table (gpu_metrics timestamp moved), overruns, tick quantiles."""
    from gpumon.config import Config
    from gpumon.monitor import GpuMonitor

    cfg = Config(backend=backend, devices=devices,
                 interval=args.capacity_interval, listen="127.0.0.1:0", http_threads=1, host="bench-node",
                 log_level="warn", fast_path=not args.no_fast_path, sample_threads=args.sample_threads,
                 rt_priority=args.rt_priority, prewarm_ms=args.prewarm_ms)
    mon = GpuMonitor(cfg, control_plane=False).start()
    try:
        if mon.start_error:
            return {"error": mon.start_error}
        mon.wait_ticks(20, timeout_s=30)  # first-tick setup (fd tables, link / RAS passes) stays out
        s0, q0, t0 = mon.ex.self_stats(), mon.ex.seq, time.perf_counter()
        time.sleep(args.capacity_s)
        s1, q1, t1 = mon.ex.self_stats(), mon.ex.seq, time.perf_counter()
        durs = [t["duration_s"] for t in mon.ex.tick_log() if q0 < t["seq"] <= q1]
    finally:
        mon.stop()
    dt = t1 - t0
    devs = max(1, len(s1.get("device_errors") or [0]))
    samples = s1["samples"] - s0["samples"]
    stale = s1.get("stale_samples", 0) - s0.get("stale_samples", 0)
    return {"interval_ms": args.capacity_interval * 1e3, "seconds": round(dt, 3), "devices": devs,
            "ticks_per_s": round((q1 - q0) / dt, 1),
            "samples_per_sec_per_gpu": round(samples / dt / devs, 1),
            # a sample whose firmware table timestamp did not move since the last tick is stale: the
            # fresh rate is bounded by how often the SMU rewrites gpu_metrics, not by the exporter
            "fresh_samples_per_sec_per_gpu": round((samples - stale) / dt / devs, 1) if has_gpu else None,
            "overruns": s1["overruns"] - s0["overruns"],
            # an overrun tick makes the sampler skip to the next interval boundary (deadline-based):
            # the back-to-back bound of the sample -> export path is 1 / the mean tick (the
            # post-publish gzip and maintenance run on the sampler thread too, outside the tick)
            "tick_bound_hz": round(len(durs) / sum(durs), 1) if durs else None,
            "tick_mean_ms": round(sum(durs) / len(durs) * 1e3, 4) if durs else None,
            "tick_p50_ms": round(_pct(durs, 0.50) * 1e3, 4) if durs else None,
            "tick_p99_ms": round(_pct(durs, 0.99) * 1e3, 4) if durs else None,
            "ticks_logged": len(durs)}


GFX_UTIL_FLOOR = 50.0  # % : a GPU the bench loads must read at least this busy in the exporter


def _device_check(rows, tick_util, loaded):
    """Each loaded GPU's exporter gfx_util, mean over the timed ticks (the first one spans the
    warmup and is skipped). A loaded GPU that reads under GFX_UTIL_FLOOR means the exporter is
    watching some other GPU: the check fails, and bench.py exits non-zero after its line."""
    ticks = tick_util[1:] if len(tick_util) > 1 else tick_util
    per = []
    for r in rows:
        xs = [t[r["index"]] for t in ticks if r["index"] < len(t) and isinstance(t[r["index"]], (int, float))
              and t[r["index"]] == t[r["index"]]]
        per.append({"hip_ordinal": r["hip_ordinal"], "gpu_id": r["gpu_id"],
                    "gfx_util_mean": round(sum(xs) / len(xs), 1) if xs else None})
    if not loaded:
        return {"ok": True, "checked": False, "reason": "no synthetic load", "per_gpu": per}
    bad = [p for p in per if p["gfx_util_mean"] is None or p["gfx_util_mean"] < GFX_UTIL_FLOOR]
    return {"ok": not bad, "checked": True, "floor_pct": GFX_UTIL_FLOOR, "per_gpu": per}


class InProcessExporter:
    """``--exporter inprocess``: the same core through gpumon._core in this process, behind the
    interface of gpumon.export.child.ChildExporter (A/B against the shipped binary)."""

    def __init__(self, mon):
        self.mon, self.ex = mon, mon.ex
        self.port = mon.port
        self.pid = os.getpid()

    @property
    def seq(self):
        return self.ex.seq

    def wait_for_seq(self, seq, timeout_s):
        return self.ex.wait_for_seq(seq, timeout_s)

    def wait_ticks(self, n=1, timeout_s=30.0):
        return self.mon.wait_ticks(n, timeout_s)

    def ticks(self, since=0):
        return [t for t in self.ex.tick_log() if t["seq"] > since]

    def scrape_count(self):
        return self.ex.scrape_count()

    def scrape_durations_since(self, n0):
        return list(self.ex.scrape_durations_since(n0))

    def statics(self):
        return self.ex.statics()

    def self_stats(self):
        return self.ex.self_stats()

    def samples(self):
        return self.ex.samples()

    def pod_rows(self):
        return self.ex.pod_rows()

    def procs(self):
        return self.ex.debug_view("/debug/procs")

    def metrics(self):
        return self.mon.metrics()

    def threads_cpu(self):
        """The exporter's own threads in this process (named gpumon-*: sampler, device workers, HTTP
        loops, pollers); the bench's loads, scraper and torch threads are not counted."""
        from gpumon.export.child import threads_cpu

        return threads_cpu(os.getpid(), "gpumon-")

    def rss_bytes(self):
        return None  # shared with the bench process: not the exporter's

    def stop(self):
        self.mon.stop()


def _cpu_quota():
    """CPUs this cgroup may use (cgroup v2 cpu.max: quota / period), None when unlimited / unknown.
    A shared GPU box gives a job a CPU share this way, not an affinity mask."""
    try:
        with open("/proc/self/cgroup") as fh:
            rel = next((l.split("::", 1)[1].strip() for l in fh if l.startswith("0::")), "/")
        with open(os.path.join("/sys/fs/cgroup", rel.lstrip("/"), "cpu.max")) as fh:
            quota, period = fh.read().split()[:2]
        return None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        return None


def _loadavg():
    try:
        with open("/proc/loadavg") as fh:
            return float(fh.read().split()[0])
    except (OSError, ValueError, IndexError):
        return None


def _per_device_times(timed, gpu_ids):
    out = []
    for i, g in enumerate(gpu_ids):
        dv = [t["dev"][i] for t in timed if i < len(t.get("dev", []))]
        if not dv:
            continue
        td = [d.get("t_device", 0.0) for d in dv]
        tp = [d.get("t_procs", 0.0) for d in dv]
        out.append({"gpu": i, "gpu_id": g, "t_device_mean_ms": round(sum(td) / len(td) * 1e3, 4),
                    "t_device_max_ms": round(max(td) * 1e3, 4), "t_procs_mean_ms": round(sum(tp) / len(tp) * 1e3, 4)})
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--interval", type=float, default=1.0, help="sampling interval (1.0 = BASELINE; 0.1 = 10 Hz stress)")
    ap.add_argument("--load", default="mixed", choices=["mixed", "concurrent", "mfma", "hbm", "idle"])
    ap.add_argument("--scrape-rate", type=float, default=200.0,
                    help="aggregate /metrics requests per second (200: >= 2000 timed scrapes in a 10 s run, "
                         "so p99 / p99.9 rest on >= 20 / 2 samples above them)")
    ap.add_argument("--scrape-concurrency", type=int, default=2)
    ap.add_argument("--gzip", action="store_true", help="scrape with Accept-Encoding: gzip")
    ap.add_argument("--scrape-path", default="/metrics",
                    help="request target, e.g. '/metrics?include=node_gpu_*,pod_gpu_*' (a per-request family filter)")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--sample-threads", type=int, default=-1,
                    help="parallel per-GPU sampling threads (-1 = auto: one per GPU, 0 = sequential)")
    ap.add_argument("--replicate", type=int, default=1,
                    help="REHEARSAL ONLY: sample each physical GPU R times (sampler scaling on a 1-GPU box)")
    ap.add_argument("--allreduce-mb", type=int, default=256, help="torchrun: all-reduce message size")
    ap.add_argument("--xgmi-duty", type=float, default=0.4,
                    help="torchrun: fraction of each interval filled with all-reduces (0 = one per step)")
    ap.add_argument("--xgmi-mb", type=int, default=256, help="single process: peer-copy ring buffer size")
    ap.add_argument("--no-xgmi", action="store_true", help="no xGMI traffic for N > 1")
    ap.add_argument("--link-check-s", type=float, default=0.6,
                    help="N > 1: seconds per peer of the GPU 0 -> k link-map check after the timed region (0 = off)")
    ap.add_argument("--probe", action="store_true", help="also run the K1 probe kernel each tick")
    ap.add_argument("--idle-s", type=float, default=-1.0,
                    help="untimed idle reference before the load starts: scrape p50/p99 + tick cost "
                         "(-1 = as long as the timed region: the same scrape count; 0 = off)")
    ap.add_argument("--idle-spinners", type=int, default=0,
                    help="DIAGNOSTIC: SCHED_IDLE busy loops during the idle reference (they take no CPU from "
                         "runnable threads but keep CPUs out of idle states: isolates wake-from-idle latency)")
    ap.add_argument("--pin-cpus", type=int, default=0,
                    help="DIAGNOSTIC: run the whole bench (exporter, scraper, loads, spinners) on the first N CPUs "
                         "of its allowed set, so --idle-spinners can keep exactly those CPUs out of idle")
    ap.add_argument("--no-fast-path", action="store_true", help="read every value through libamd_smi")
    ap.add_argument("--rt-priority", type=int, default=1,
                    help="the DaemonSet's rt_priority (SCHED_FIFO sampler; stays normal without CAP_SYS_NICE)")
    ap.add_argument("--http-rt-priority", type=int, default=1,
                    help="the DaemonSet's http_rt_priority (SCHED_FIFO HTTP loops; normal without CAP_SYS_NICE)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise torch.distributed (RCCL) even with one rank: rehearses the torchrun path "
                         "(process group, barriers, MAX over ranks) on a 1-GPU box")
    ap.add_argument("--prewarm-ms", type=float, default=3.0,
                    help="device workers warm the firmware-table path this long before each tick (0 = off)")
    ap.add_argument("--capacity-s", type=float, default=2.0,
                    help="untimed sampler-capacity run after the timed region (seconds; 0 = off)")
    ap.add_argument("--capacity-interval", type=float, default=0.001,
                    help="sampling interval of the capacity run (seconds)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="DIAGNOSTIC: extra exporter config keys for the timed exporter (gpumon.config.Config), "
                         "e.g. --set processes=false --set gzip=false; listed in the line as exporter_overrides")
    ap.add_argument("--ranks-per-gpu", type=int, default=1,
                    help="REHEARSAL on a box with fewer GPUs: K torchrun ranks share each GPU (gloo process group, "
                         "no xGMI traffic); the line's data and parallelism say so")
    ap.add_argument("--exporter", default="child", choices=["child", "inprocess"],
                    help="child: bin/gpumon-exporter as its own process (the shipped binary, default); "
                         "inprocess: the same core through gpumon._core in this process (A/B)")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    if args.idle_s < 0:
        args.idle_s = max(5.0, args.steps * args.interval)
    if args.pin_cpus > 0:  # before any thread exists: every thread and child inherits the mask
        os.sched_setaffinity(0, sorted(os.sched_getaffinity(0))[:args.pin_cpus])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    rpg = max(1, args.ranks_per_gpu)
    if world > 1 and world % rpg:
        raise SystemExit(f"--ranks-per-gpu {rpg} does not divide the world size {world}")
    n = max(1, args.gpus if world == 1 else world // rpg)

    try:
        import torch
    except ImportError:  # a lean image (the exporter's + tools): one process, the native HIP path only
        torch = None
        if world > 1:
            raise SystemExit("bench.py under torchrun needs PyTorch (torch.distributed over RCCL)")

    # torchrun: this rank's GPU; one process: all N GPUs (the node-level exporter watches them all)
    my_devs = [local_rank // rpg] if world > 1 else list(range(n))

    # ---------------------------------------------------------------- rank 0: the exporter child
    # Started BEFORE this process's first HIP call (torch.cuda.is_available() initialises HIP): the
    # child is forked from a process without GPU state. The loaded GPUs' BDFs come from KFD's
    # topology here (devmap.kfd_bdfs) and are checked against HIP's after initialisation.
    from gpumon.parallel.devmap import kfd_bdfs

    predicted = kfd_bdfs(range(n)) if rank == 0 else {}
    gpu_guess = (torch.cuda.device_count() > 0) if torch is not None else bool(kfd_bdfs(range(1)))
    backend = args.backend
    if backend == "auto":
        # auto = libamd_smi with the sysfs fast path, rocm_smi_lib if libamd_smi cannot initialise
        backend = "auto" if gpu_guess else f"mock:gpus={n * args.replicate},mode=load"
        if gpu_guess and args.replicate > 1:
            backend = f"amdsmi:replicate={args.replicate}"
    real = backend.startswith(("amdsmi", "rocm_smi", "auto"))
    overrides = dict(kv.split("=", 1) for kv in args.set)
    ex = None
    exporter_info = {"mode": args.exporter}
    if rank == 0 and args.exporter == "child":
        import tempfile

        from gpumon.export.child import ChildExporter, daemonset_config

        sampled = [predicted[k] for k in range(n)] if real and len(predicted) == n else []
        ccfg = dict(daemonset_config(), backend=backend, devices=sampled, interval=args.interval, host="bench-node",
                    http_threads=2, http_rt_priority=args.http_rt_priority, rt_priority=args.rt_priority,
                    prewarm_ms=args.prewarm_ms, sample_threads=args.sample_threads,
                    fast_path=not args.no_fast_path, enable_probe=bool(args.probe and gpu_guess), log_level="warn",
                    **overrides)
        workdir = tempfile.mkdtemp(prefix="gpumon-bench-")
        ex = ChildExporter(ccfg, workdir).start()
        exporter_info.update(binary="bin/gpumon-exporter", pid=ex.pid, config_keys=sorted(ccfg),
                             spawned_before_hip=True, devices_predicted=sampled)

    if torch is not None:
        has_gpu = torch.cuda.is_available()
    else:
        from gpumon import hip as _hip_rt

        has_gpu = _hip_rt().device_count() > 0
    dist = None
    if world > 1 or (args.dist and torch is not None):
        import torch.distributed as dist

        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29517"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)  # --dist without a launcher
        if has_gpu:
            torch.cuda.set_device(my_devs[0])
        # RCCL takes one rank per GPU; ranks sharing a GPU (the rehearsal) reduce over gloo
        dist.init_process_group(backend="nccl" if has_gpu and rpg == 1 else "gloo")
    device = (torch.device(f"cuda:{my_devs[0]}") if has_gpu else torch.device("cpu")) if torch is not None else None
    # where this rank's small reductions (timings, rates) live: the GPU under RCCL, else the host
    red_device = None
    if torch is not None:
        red_device = device if dist is not None and dist.get_backend() == "nccl" else torch.device("cpu")

    # HIP ordinal -> PCI BDF of every GPU the job loads, gathered to rank 0: the exporter samples
    # exactly those GPUs, named by BDF, since its gpu_id (libamd_smi hip_id) is node-wide and a
    # HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES subset renumbers the ordinals (devmap.py)
    ord_bdfs = {}
    if has_gpu:
        from gpumon.parallel.devmap import hip_bdfs

        ord_bdfs = hip_bdfs(my_devs)
        if dist is not None:
            allb = [None] * world
            dist.all_gather_object(allb, ord_bdfs)
            ord_bdfs = {int(k): v for d in allb for k, v in d.items()}
    # every rank's view of the process group (SCALE: RCCL's world size as each rank sees it) and its
    # pid (the tenants the exporter attributes)
    ranks_seen = [{"rank": rank, "world_size": dist.get_world_size() if dist is not None else 1,
                   "backend": str(dist.get_backend()) if dist is not None else None, "pid": os.getpid(),
                   "local_rank": local_rank, "device": my_devs[0] if world > 1 else None}]
    if dist is not None:
        allr = [None] * world
        dist.all_gather_object(allr, ranks_seen[0])
        ranks_seen = allr

    def barrier():
        if dist is not None:
            dist.barrier()
        if has_gpu and torch is not None:
            torch.cuda.synchronize()

    # ---------------------------------------------------------------- rank 0: exporter + scraper
    core = None
    mon = None
    sampled = [ord_bdfs[k] for k in sorted(ord_bdfs)] if real and ord_bdfs else []
    if rank == 0:
        from gpumon import core as _core
        from gpumon.parallel.devmap import DeviceMapError, match, positional

        core = _core()
        if ex is None:  # --exporter inprocess
            from gpumon.config import Config
            from gpumon.monitor import GpuMonitor

            cfg = Config(backend=backend, devices=sampled,
                         interval=args.interval, listen="127.0.0.1:0", http_threads=2, host="bench-node",
                         http_rt_priority=args.http_rt_priority,
                         enable_probe=args.probe and has_gpu, log_level="warn", fast_path=not args.no_fast_path,
                         sample_threads=args.sample_threads, rt_priority=args.rt_priority, prewarm_ms=args.prewarm_ms)
            if overrides:
                cfg.apply_dict(overrides)
            mon = GpuMonitor(cfg, control_plane=False).start()
            if mon.start_error:
                raise SystemExit(f"exporter backend failed: {mon.start_error}")
            ex = InProcessExporter(mon)
            exporter_info.update(binary=None, pid=os.getpid())

        def pair():
            st = ex.statics()
            if len(st) < n:
                raise DeviceMapError(f"exporter sees {len(st)} GPU(s), bench needs {n}")
            return (match(ord_bdfs, st, replicas=args.replicate > 1) if real and ord_bdfs else positional(n, st))

        try:  # every loaded ordinal paired with the exporter device of the same BDF
            dev_rows = pair()
        except DeviceMapError as e:
            if args.exporter != "child" or not sampled:
                raise SystemExit(f"bench: loaded GPUs and sampled GPUs disagree: {e}")
            # the KFD-topology prediction missed (an unusual visibility setup): the child starts
            # again with HIP's own BDFs, now after HIP initialised, and the line says so
            ex.stop()
            ex = ChildExporter(dict(ex.cfg, devices=sampled), ex.workdir).start()
            exporter_info.update(pid=ex.pid, spawned_before_hip=False, respawned_after=str(e))
            try:
                dev_rows = pair()
            except DeviceMapError as e2:
                raise SystemExit(f"bench: loaded GPUs and sampled GPUs disagree: {e2}")
        if backend == "auto":
            backend = ex.self_stats().get("backend") or backend  # the one that came up
        exporter_info["devices_match_hip"] = (sampled == exporter_info.get("devices_predicted", sampled))

    # ---------------------------------------------------------------- idle reference (untimed)
    # the same scrape load against the same exporter before any synthetic load starts: the
    # BASELINE asks for scrape p99 idle and under load at every GPU count
    idle = None
    if rank == 0 and args.idle_s > 0:
        ex.wait_ticks(1, timeout_s=args.interval * 5 + 30)
        spin = []
        if args.idle_spinners > 0:
            import subprocess

            code = "import os; os.sched_setscheduler(0, os.SCHED_IDLE, os.sched_param(0))\nwhile True: pass"
            spin = [subprocess.Popen([sys.executable, "-c", code]) for _ in range(args.idle_spinners)]
            time.sleep(1.0)
        q0 = ex.seq
        n0 = ex.scrape_count()
        try:
            r = core.scrape_load("127.0.0.1", ex.port, args.scrape_path, n_requests=0, duration_s=args.idle_s,
                                 concurrency=args.scrape_concurrency, rate_hz=args.scrape_rate, keep_alive=True,
                                 gzip=args.gzip)
        finally:
            for p in spin:
                p.kill()
                p.wait()
        q1 = ex.seq
        it = [t["duration_s"] for t in ex.ticks(q0) if q0 < t["seq"] <= q1]
        lat = r.get("latencies_s", [])
        srv = _server_durations(ex, n0, len(lat))
        idle = {"seconds": args.idle_s, "scrapes": len(lat), "scrape_errors": r.get("errors", 0),
                "scrape_p50_ms": round(_pct(lat, 0.50) * 1e3, 4) if lat else None,
                "scrape_p99_ms": round(_pct(lat, 0.99) * 1e3, 4) if lat else None,
                "scrape_p999_ms": round(_pct(lat, 0.999) * 1e3, 4) if lat else None,
                "scrape_p99_ci95_ms": _ci(lat, 0.99),
                "server_scrape_p99_ms": round(_pct(srv, 0.99) * 1e3, 4) if srv else None,
                "server_scrape_p999_ms": round(_pct(srv, 0.999) * 1e3, 4) if srv else None,
                "ticks": len(it), "tick_mean_ms": round(sum(it) / len(it) * 1e3, 4) if it else None,
                "tick_max_ms": round(max(it) * 1e3, 4) if it else None,
                "idle_spinners": args.idle_spinners,
                "pinned_cpus": sorted(os.sched_getaffinity(0)) if args.pin_cpus > 0 else None}
    barrier()

    # ---------------------------------------------------------------- synthetic load on every GPU
    loads = []
    if has_gpu and args.load != "idle":
        from gpumon import hip
        from gpumon.ops.load import SyntheticLoad

        if hip().device_count() < max(my_devs) + 1:
            raise SystemExit(f"bench needs GPUs {my_devs}, HIP sees {hip().device_count()}")
        loads = [SyntheticLoad(dev=d, kind=args.load, hbm_bytes=1 << 30).start() for d in my_devs]

    xgmi_on = n > 1 and rpg == 1 and not args.no_xgmi
    ar_buf = None
    if dist is not None and xgmi_on and args.allreduce_mb > 0:
        # zeros: repeated in-place sums stay finite (ones would reach inf after ~40 steps on 8 ranks)
        ar_buf = torch.zeros(args.allreduce_mb * (1 << 20) // 2, dtype=torch.bfloat16, device=device)
    copiers = []
    if dist is None and has_gpu and xgmi_on:
        from gpumon.parallel.xgmi import PeerCopier

        copiers = [PeerCopier(i, (i + 1) % n, nbytes=args.xgmi_mb << 20).start() for i in range(n)]

    if rank == 0:
        ex.wait_ticks(args.warmup, timeout_s=args.warmup * args.interval * 5 + 30)
    barrier()
    # RCCL channel / buffer setup and the all-reduce calibration stay out of the timed region
    reps = 1
    ar_cal_ms = None
    if ar_buf is not None:
        for _ in range(3):
            dist.all_reduce(ar_buf)
        if has_gpu:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                dist.all_reduce(ar_buf)
            e1.record()
            e1.synchronize()
            t = torch.tensor([e0.elapsed_time(e1) / 5], dtype=torch.float64, device=red_device)
        else:
            t0 = time.perf_counter()
            for _ in range(5):
                dist.all_reduce(ar_buf)
            t = torch.tensor([(time.perf_counter() - t0) / 5 * 1e3], dtype=torch.float64, device=red_device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # every rank derives the same count
        ar_cal_ms = float(t.item())
        if args.xgmi_duty > 0 and ar_cal_ms > 0:
            reps = max(1, min(4000, int(args.xgmi_duty * args.interval * 1e3 / ar_cal_ms)))

    scrape_result = {}
    scraper = None
    if rank == 0:
        # Start the timed region right after a tick: the K timed ticks then close K whole intervals
        # (t0 + I, ..., t0 + K*I), whatever the calibration above took. Each step's all-reduces run
        # INSIDE its interval, before the tick that closes it, so the region ends at tick K -- not
        # a random phase of an interval plus the last step's reductions past it (the elapsed time
        # then moved by up to -0.6 / +0.4 intervals with the phase, i.e. +-4-6 % of a 10-step
        # samples/s, at N > 1 only).
        ex.wait_ticks(1, timeout_s=args.interval * 5 + 30)
        duration = args.steps * args.interval

        def _scrape():
            scrape_result.update(core.scrape_load("127.0.0.1", ex.port, args.scrape_path, n_requests=0,
                                                  duration_s=duration, concurrency=args.scrape_concurrency,
                                                  rate_hz=args.scrape_rate, keep_alive=True, gzip=args.gzip))

        scraper = threading.Thread(target=_scrape, daemon=True)
        n_scr0 = ex.scrape_count()
        s0 = ex.self_stats()
        seq0 = ex.seq
        cpu0 = ex.threads_cpu()

    # ---------------------------------------------------------------- timed region
    barrier()
    load_before = _loadavg()
    c0 = [c.stats() for c in copiers]
    l0 = [ld.stats() for ld in loads]
    t0 = time.perf_counter()
    if scraper is not None:
        scraper.start()
    ar_events = []
    for step in range(args.steps):
        # one step = one sampling interval: this interval's xGMI traffic, then the tick closing it
        if ar_buf is not None:
            if has_gpu:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
                for _ in range(reps):
                    dist.all_reduce(ar_buf)
                ev[1].record()
                ar_events.append(ev)
            else:
                for _ in range(reps):
                    dist.all_reduce(ar_buf)
        if rank == 0:
            if not ex.wait_for_seq(seq0 + step + 1, args.interval * 5 + 10):
                raise SystemExit("exporter tick timed out")
    barrier()
    elapsed = time.perf_counter() - t0
    if rank == 0:  # the exporter's counters at the end of the timed region (not after the reductions)
        s1 = ex.self_stats()
        seq1 = ex.seq
        cpu1 = ex.threads_cpu()
    c1 = [c.stats() for c in copiers]
    l1 = [ld.stats() for ld in loads]
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---------------------------------------------------------------- per-GPU load rates (every rank)
    # event-timed TFLOP/s / TB/s over the timed region, gathered to rank 0 as one row per GPU
    lrates = [[0.0, 0.0, 0.0] for _ in range(n)]
    for d, a, b in zip(my_devs, l0, l1):
        from gpumon.ops.load import SyntheticLoad

        r = SyntheticLoad.rates(a, b)
        # ranks sharing a GPU: the work over wall time adds up to the GPU's; rates over each
        # process's own kernel time do not (its MFMA batches overlap another's HBM batches)
        lrates[d] = [r["tflops_wall"], r["tbps_wall"], r["busy"]] if rpg > 1 else [r["tflops"], r["tbps"], r["busy"]]
    if dist is not None:
        t = torch.tensor(lrates, dtype=torch.float64, device=red_device)
        dist.all_reduce(t)
        lrates = t.cpu().tolist()

    # ---------------------------------------------------------------- xGMI expectation
    xgmi = None
    exp_tx = exp_rx = None
    if ar_buf is not None:
        nbytes = ar_buf.numel() * ar_buf.element_size()
        ar_ms = [a.elapsed_time(b) / reps for a, b in ar_events] if ar_events else []
        t = torch.tensor([sum(ar_ms) / len(ar_ms) if ar_ms else float("nan")], dtype=torch.float64,
                         device=red_device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ar_mean_s = float(t.item()) * 1e-3
        per_gpu = 2 * (n - 1) / n * nbytes * reps * args.steps / elapsed  # B/s out of (and into) every GPU
        exp_tx = exp_rx = [per_gpu] * n
        xgmi = {"mode": "rccl_allreduce", "allreduce_mb": args.allreduce_mb, "allreduces_per_step": reps,
                "calibration_ms": _r(ar_cal_ms),
                "allreduce_ms": round(ar_mean_s * 1e3, 3) if ar_mean_s == ar_mean_s else None,
                "allreduce_busbw_GBps": round(2 * (n - 1) / n * nbytes / ar_mean_s / 1e9, 2)
                if ar_mean_s == ar_mean_s and ar_mean_s > 0 else None,
                "expected_tx_GBps_per_gpu": round(per_gpu / 1e9, 3)}
    elif copiers:
        rates = [(b["bytes"] - a["bytes"]) / max(1e-9, b["wall_s"] - a["wall_s"]) for a, b in zip(c0, c1)]
        exp_tx = rates
        exp_rx = [rates[(d - 1) % n] for d in range(n)]
        xgmi = {"mode": "peer_copy_ring", "copy_mb": args.xgmi_mb,
                "copy_GBps": [round(r / 1e9, 2) for r in rates],
                "expected_tx_GBps_per_gpu": round(sum(rates) / n / 1e9, 3)}
    for c in copiers:
        c.close()

    result = None
    if rank == 0:
        if scraper is not None:
            scraper.join(timeout=args.interval * 5 + 30)
        lat = scrape_result.get("latencies_s", [])
        srv = _server_durations(ex, n_scr0, len(lat))  # server-side, the same scrapes
        ticks = seq1 - seq0
        timed = [t for t in ex.ticks(seq0) if seq0 < t["seq"] <= seq0 + ticks]
        # per tick, per sampled device: (sum of per-link write B/s, read B/s) or None, and gfx_util:
        # every timed tick's values from the exporter's tick log (none raced for)
        tick_rates = [[(d["xgmi_wr_Bps"] or 0.0, d["xgmi_rd_Bps"] or 0.0) if d.get("rates_valid") else None
                       for d in t.get("dev", [])] for t in timed]
        tick_util = [[d.get("gfx_util") for d in t.get("dev", [])] for t in timed]
        samples = s1["samples"] - s0["samples"]
        stale = s1.get("stale_samples", 0) - s0.get("stale_samples", 0)
        # value: fresh samples (the firmware table advanced) of the LOADED GPUs over the timed ticks
        idx = [r["index"] for r in dev_rows]
        fresh = sum(1 for t in timed for i in idx
                    if i < len(t.get("dev", [])) and t["dev"][i].get("ok") and t["dev"][i].get("fresh"))
        tdur = [t["duration_s"] for t in timed]
        slow = max(timed, key=lambda t: t["duration_s"]) if timed else None
        sm = ex.samples()
        util = [x["fields"].get("gfx_util") for x in sm]
        rows = ex.pod_rows()
        value = fresh / elapsed
        check = _device_check(dev_rows, tick_util, loaded=bool(loads) and args.load != "idle")
        from gpumon.export import promtext

        gid = {r["hip_ordinal"]: r["gpu_id"] for r in dev_rows}
        fam = promtext.parse(ex.metrics())
        slot_map = {}  # xGMI link-metrics entry -> table slot pairing (csrc/core/xgmi_map.cpp)
        for what in ("verified", "unverified", "mismatch"):
            for _, lab, v in fam.get(f"gpumon_xgmi_slot_map_{what}", {}).get("samples", []):
                slot_map.setdefault(lab.get("gpu_id"), {})[what] = int(v)
        # rows per GPU: a multi-rank tenant's ranks open every GPU; the first 8-GPU
        # record must show whether each GPU carries one workload row (peer contexts hidden) or N
        active = {lab.get("gpu_id"): int(v) for _, lab, v in fam.get("gpu_active_processes", {}).get("samples", [])}
        stat_ids = [st.get("gpu_id", str(i)) for i, st in enumerate(ex.statics())]
        per_gpu_rows = []
        for i, g in enumerate(stat_ids):
            wr = [r for r in rows if not r["idle"] and r["dev"] == i]
            per_gpu_rows.append({"gpu": i, "gpu_id": g, "rows": len(wr), "pids": sorted(r["pid"] for r in wr)[:8],
                                 "idle_rows": sum(1 for r in rows if r["idle"] and r["dev"] == i),
                                 "active_processes": active.get(g)})
        # the contexts behind hidden_contexts / hidden_peer_contexts, by pid, with the exporter's
        # reason: "empty" (no VRAM, no waves: a runtime that only opened the GPU), "peer" (a
        # multi-GPU process's context on a GPU it does no work on), "helper", "not opted in"
        ctx = ex.procs()
        hidden_detail = [{"gpu": c["dev"], "pid": c["pid"], "queues": c["queues"],
                          "vram_mib": round(c["vram_bytes"] / 2 ** 20, 1) if c["vram_bytes"] is not None else None,
                          "why": c["why"]}
                         for c in ctx if not c["row"]][:16]
        hidden_reasons = {}
        for c in ctx:
            if not c["row"]:
                hidden_reasons[c["why"]] = hidden_reasons.get(c["why"], 0) + 1
        rows_per_user = {}
        for r in rows:
            rows_per_user[r["user_name"]] = rows_per_user.get(r["user_name"], 0) + 1
        per_gpu = _per_gpu_xgmi(tick_rates, dev_rows, exp_tx, exp_rx) if xgmi is not None else None
        if xgmi is not None:
            tx = [r["exporter_tx_GBps"] for r in per_gpu if r["exporter_tx_GBps"] is not None]
            rx = [r["exporter_rx_GBps"] for r in per_gpu if r["exporter_rx_GBps"] is not None]
            xgmi["exporter_tx_GBps_per_gpu"] = round(sum(tx) / len(tx), 3) if tx else None
            xgmi["exporter_rx_GBps_per_gpu"] = round(sum(rx) / len(rx), 3) if rx else None
            if tx and xgmi.get("expected_tx_GBps_per_gpu"):
                xgmi["exporter_vs_expected"] = round(xgmi["exporter_tx_GBps_per_gpu"]
                                                     / xgmi["expected_tx_GBps_per_gpu"], 3)
            if rx and xgmi.get("expected_tx_GBps_per_gpu"):  # a ring moves as much in as out
                # RCCL may push (writes: tx) or pull (reads: rx); the receive side is reported too
                xgmi["exporter_rx_vs_expected"] = round(xgmi["exporter_rx_GBps_per_gpu"]
                                                        / xgmi["expected_tx_GBps_per_gpu"], 3)
            xgmi["per_gpu"] = per_gpu
        # the exporter's CPU over the timed region, per thread name (millicores) and in total
        thr = {k: round(1000.0 * (v - cpu0.get(k, 0.0)) / elapsed, 2) for k, v in sorted(cpu1.items())}
        tenant_pids = sorted({x["pid"] for x in ranks_seen})
        row_pids = sorted({int(r["pid"]) for r in rows if not r["idle"] and str(r["pid"]).isdigit()})
        # KFD lists HOST pids: in a container with its own pid namespace (a gpurun box) the rows
        # carry pids this process cannot see, and the tenants are checked by count instead -- one
        # workload row per loaded GPU per rank on it, none of them the exporter's
        same_ns = bool(set(row_pids) & set(tenant_pids))
        want_rows = {r["index"]: sum(1 for x in ranks_seen if world == 1 or x["device"] == r["hip_ordinal"])
                     for r in dev_rows}
        got_rows = {r["index"]: sum(1 for x in rows if not x["idle"] and x["dev"] == r["index"]) for r in dev_rows}
        exporter_info.update(
            rss_mb=round(ex.rss_bytes() / 2 ** 20, 1) if ex.rss_bytes() else None,
            tenant_pids=tenant_pids,
            row_pids=row_pids,
            pid_namespace="shared" if same_ns else "separate (rows carry host pids)",
            # in a cluster the exporter only ever attributes other processes: every pod row is a
            # tenant's (by pid where the namespaces agree, else by count), none the exporter's own
            rows_are_tenants=(set(row_pids) <= set(tenant_pids) if same_ns else got_rows == want_rows)
            if has_gpu and loads else None,
            exporter_pid_in_rows=exporter_info.get("pid") in row_pids)
        result = {
            "metric": BASELINE_METRIC,
            "value": round(value, 4),
            "unit": "samples/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / max(1, len(dev_rows)) / BASELINE_SAMPLES_PER_GPU, 3),
            "value_note": ("value = fresh samples/s of the loaded GPUs over the timed ticks (samples whose firmware "
                           "table advanced; repeats of the last table are not counted): fixed by the sampling "
                           "interval (1/interval per GPU) unless ticks overrun or the interval beats the SMU's "
                           "refresh; the measured speed is scrape_p99_ms / scrape_p999_ms (client), "
                           "server_scrape_p99_ms and tick_*_ms"),
            "samples_total": samples,
            "stale_samples": stale,
            "dtype": "bf16",
            "data": (f"synthetic (REHEARSAL: {world} ranks share {n} GPU(s), gloo process group, no xGMI traffic)"
                     if rpg > 1 and has_gpu else
                     "synthetic" if backend in ("amdsmi", "rocm_smi") else
                     f"synthetic (REHEARSAL: {n} physical GPU(s) each sampled {args.replicate}x)"
                     if backend.startswith("amdsmi:replicate") else "synthetic (mock backend: no GPU visible)"),
            "exporter": exporter_info.get("binary") or "in-process (gpumon._core)",
            "exporter_pid": exporter_info.get("pid"),
            "exporter_info": exporter_info,
            "sampled_devices": len(sm),
            # each loaded HIP ordinal and the exporter device sampled for it (same PCI BDF)
            "devices": [{k: r[k] for k in ("hip_ordinal", "bdf", "gpu_id")} for r in dev_rows],
            "device_check": check,
            "ranks": ranks_seen,
            "config": {
                "model": f"gpumon MI355X exporter ({backend.split(':')[0]} backend) + synthetic bf16 MFMA/HBM HIP load",
                "global_batch": n,
                "seq_len": None,
                "parallelism": f"node-local exporter over {n} GPU(s); "
                               + ((f"{rpg} ranks per GPU (rehearsal)" if rpg > 1 else "one rank per GPU")
                                  if world > 1 else "one process loading every GPU")
                               + (f", {'RCCL' if has_gpu else 'gloo'} all-reduce x{reps} per step"
                                  if ar_buf is not None else "")
                               + (", peer-copy xGMI ring" if copiers else ""),
                "interval_s": args.interval,
            },
            "scrape_idle": idle,  # same scrape load, before any synthetic load (untimed)
            "scrape_p50_ms": round(_pct(lat, 0.50) * 1e3, 4),
            "scrape_p99_ms": round(_pct(lat, 0.99) * 1e3, 4),
            "scrape_p999_ms": round(_pct(lat, 0.999) * 1e3, 4),
            "scrape_p99_ci95_ms": _ci(lat, 0.99),
            "scrape_max_ms": round(max(lat) * 1e3, 4) if lat else None,
            "scrapes": len(lat),
            "scrape_rate_hz": args.scrape_rate,
            "scrape_path": args.scrape_path,
            # the exporter's own service time of the same requests (request parsed -> response
            # written), exact: client minus server = loopback + client scheduling
            "server_scrape_p50_ms": round(_pct(srv, 0.50) * 1e3, 4) if srv else None,
            "server_scrape_p99_ms": round(_pct(srv, 0.99) * 1e3, 4) if srv else None,
            "server_scrape_p999_ms": round(_pct(srv, 0.999) * 1e3, 4) if srv else None,
            "server_scrapes": len(srv),
            "scrape_errors": scrape_result.get("errors", 0),
            "scrape_body_kb": round(scrape_result.get("bytes", 0) / max(1, len(lat)) / 1024, 2),
            "samples_per_sec_per_gpu": round(value / max(1, len(dev_rows)), 4),
            "ticks": ticks,
            "tick_mean_ms": round(sum(tdur) / len(tdur) * 1e3, 4) if tdur else None,
            "tick_p50_ms": round(_pct(tdur, 0.50) * 1e3, 4) if tdur else None,
            "tick_p99_ms": round(_pct(tdur, 0.99) * 1e3, 4) if tdur else None,
            "tick_max_ms": round(max(tdur) * 1e3, 4) if tdur else None,
            # what the slowest timed tick spent its time on (tick-tail attribution)
            "slowest_tick": {k: (round(v * 1e3, 4) if k.startswith("t_") or k == "duration_s" else v)
                             for k, v in slow.items() if k in ("seq", "duration_s", "t_late", "t_sample", "t_wake", "t_device",
                                                               "t_procs", "t_attrib", "t_render", "t_gzip",
                                                               "link_refreshes", "ras_reads", "ras_full")} if slow else None,
            # mean phase times over the timed ticks (ms): where a typical tick goes
            "tick_phases_mean_ms": {k: round(sum(t[k] for t in timed) / len(timed) * 1e3, 4)
                                    for k in ("t_late", "t_sample", "t_wake", "t_device", "t_procs", "t_attrib",
                                              "t_render", "t_gzip")} if timed else None,
            # per sampled device: its own calls' time per tick (the worker's metrics + links + RAS +
            # process list, and the process list alone), mean / max over the timed ticks (ms)
            "per_device_tick_ms": _per_device_times(timed, stat_ids),
            "tick_quantiles": "exact over the timed ticks (exporter tick log); times in ms",
            "overruns": s1["overruns"] - s0["overruns"],
            "sampler_rt_threads": s1.get("rt_threads", 0),
            "http_rt_loops": s1.get("http_rt_loops"),
            "prewarm_ms": args.prewarm_ms,
            "exporter_overrides": args.set or None,
            # the exporter's own threads over the timed region, serving the scrape load too
            "exporter_cpu_millicores": round(sum(thr.values()), 2),
            "exporter_thread_cpu_millicores": thr,
            "backend_call_us": {k: round((v["seconds"] - s0["backend_calls"].get(k, {}).get("seconds", 0.0)) * 1e6
                                         / max(1, v["n"] - s0["backend_calls"].get(k, {}).get("n", 0)), 1)
                                for k, v in s1.get("backend_calls", {}).items()},
            "backend": backend,
            "load": args.load if has_gpu else "none",
            "load_rates": ("work over wall time, summed over the ranks sharing each GPU" if rpg > 1 else
                           "TFLOP/s over the MFMA batches' GPU time, TB/s over the HBM batches' GPU time"),
            "load_per_gpu": [{"gpu": d, "gpu_id": gid.get(d), "tflops": round(r[0], 1), "tbps": round(r[1], 3),
                              "busy": round(r[2], 3)}
                             for d, r in enumerate(lrates)] if has_gpu and loads else None,
            "load_tflops": round(sum(r[0] for r in lrates), 1) if has_gpu and loads else None,
            "load_tbps": round(sum(r[1] for r in lrates), 3) if has_gpu and loads else None,
            "gfx_util_last": util,
            "procs_seen": len([r for r in rows if not r["idle"]]),
            "proc_rows": [{"gpu": r["dev"], "pid": r["pid"], "vram_gib": round(r["used_memory_bytes"] / 2 ** 30, 2),
                           "cu_occupancy": _r(r["cu_occupancy"], 1), "occ_samples": r["occ_samples"],
                           "busy_pct": _r(r["proc_gfx_util"], 1)}
                          for r in rows if not r["idle"]][:16],
            "occupancy_reads": s1.get("occupancy_reads", 0) - s0.get("occupancy_reads", 0),
            "per_gpu_rows": per_gpu_rows,
            "rows_per_user": rows_per_user,
            "hidden_contexts": s1.get("hidden_contexts"),
            "hidden_peer_contexts": s1.get("hidden_peer_contexts"),
            "hidden_context_detail": hidden_detail,  # the first 16
            "hidden_context_reasons": hidden_reasons,
            "xgmi": xgmi,
            "xgmi_slot_map": slot_map or None,
            "reference_samples_per_sec_per_gpu": BASELINE_SAMPLES_PER_GPU,
            # the host around the timed region (a shared box's other jobs show here: client-side
            # tails on a busy host are its scheduling, not the exporter's service time)
            "host_load": {"loadavg_1m_before": load_before, "loadavg_1m_after": _loadavg(),
                          "cpus_usable": len(os.sched_getaffinity(0)), "cpus_host": os.cpu_count(),
                          "cpu_quota": _cpu_quota()},
        }
        rc_child = ex.stop()
        if args.exporter == "child" and rc_child == 0:  # a clean exit: its config and log go too
            import shutil

            shutil.rmtree(ex.workdir, ignore_errors=True)
        if has_gpu and n > 1 and args.link_check_s > 0:
            # validation evidence, never a reason to lose the measured line: errors and a stuck
            # peer copy are recorded, not raised (each pair runs link_check_s plus the exporter's
            # start-up; the bound leaves several times that)
            lm = _bounded(_link_map_check, 30 + (n - 1) * (4 * args.link_check_s + 5), ord_bdfs, args.link_check_s)
            result["xgmi"] = dict(result["xgmi"] or {}, link_map=lm)
        if args.capacity_s > 0:
            result["capacity"] = _bounded(_capacity, 60 + 4 * args.capacity_s, backend, sampled, args, has_gpu)
    if result is not None:  # the line is out before the teardown collectives can stall on a peer
        line = json.dumps(result)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as fh:
                fh.write(line + "\n")
    for ld in loads:
        ld.stop()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if result is not None and not result["device_check"]["ok"]:
        print(f"bench: FAILED device check: {json.dumps(result['device_check'])}", file=sys.stderr, flush=True)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
