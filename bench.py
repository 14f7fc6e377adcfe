#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): p99 /metrics scrape latency + samples/sec/GPU at 1 Hz.

    python bench.py [--gpus N --steps K --warmup W]                       # 1 GPU
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W           # N GPUs, one rank each

What one "step" is: one sampling period of the exporter (default 1 Hz, the BASELINE interval).
Rank 0 runs the native exporter (amdsmi backend) over GPUs 0..N-1 and a client-side scraper that
hits /metrics at --scrape-rate while every rank keeps its own GPU under a synthetic gfx950 HIP load
(bf16 MFMA burn + HBM stream, csrc/hip/kernels.hip) and, for N > 1, runs one RCCL all-reduce per
step (xGMI traffic). W warmup ticks, then exactly K ticks are timed between barriers +
torch.cuda.synchronize(); the MAX elapsed over ranks is used.

Reported ``value`` = whole-node fresh device samples per second (K ticks x N GPUs / elapsed);
``vs_baseline`` = per-GPU rate / 0.077 samples/s/GPU, the reference's best observed rate
(one node_gpu line per 13-19 s). The scrape-latency half of the headline metric is
reported as ``scrape_p99_ms`` / ``scrape_p50_ms`` (client-side, keep-alive, like a Prometheus
server). Without a GPU the exporter uses the mock backend and says so in ``data``.
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


def _xgmi_summary(xgmi, xgmi_rates):
    """Exporter-measured xGMI traffic over the timed ticks (mean per GPU), next to the all-reduce
    expectation. The first tick's rate spans part of the warmup, so it is skipped."""
    ticks = [t for t in xgmi_rates[1:] if t] or [t for t in xgmi_rates if t]
    out = dict(xgmi or {})
    if ticks:
        tx = [sum(w for w, _ in t) / len(t) for t in ticks]
        rx = [sum(r for _, r in t) / len(t) for t in ticks]
        out["exporter_tx_GBps_per_gpu"] = round(sum(tx) / len(tx) / 1e9, 3)
        out["exporter_rx_GBps_per_gpu"] = round(sum(rx) / len(rx) / 1e9, 3)
        exp = out.get("expected_tx_GBps_per_gpu")
        if exp:
            out["exporter_vs_expected"] = round(out["exporter_tx_GBps_per_gpu"] / exp, 3)
    return out or None


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--interval", type=float, default=1.0, help="sampling interval (1.0 = BASELINE; 0.1 = 10 Hz stress)")
    ap.add_argument("--load", default="mixed", choices=["mixed", "mfma", "hbm", "idle"])
    ap.add_argument("--scrape-rate", type=float, default=20.0, help="aggregate /metrics requests per second")
    ap.add_argument("--scrape-concurrency", type=int, default=2)
    ap.add_argument("--gzip", action="store_true", help="scrape with Accept-Encoding: gzip")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--sample-threads", type=int, default=-1,
                    help="parallel per-GPU sampling threads (-1 = auto: one per GPU, 0 = sequential)")
    ap.add_argument("--replicate", type=int, default=1,
                    help="REHEARSAL ONLY: sample each physical GPU R times (sampler scaling on a 1-GPU box)")
    ap.add_argument("--allreduce-mb", type=int, default=256)
    ap.add_argument("--probe", action="store_true", help="also run the K1 probe kernel each tick")
    ap.add_argument("--no-fast-path", action="store_true", help="read every value through libamd_smi")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n = max(1, args.gpus if world == 1 else world)

    import torch

    has_gpu = torch.cuda.is_available()
    dist = None
    if world > 1:
        import torch.distributed as dist

        if has_gpu:
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl" if has_gpu else "gloo")
    device = torch.device(f"cuda:{local_rank}") if has_gpu else torch.device("cpu")

    def barrier():
        if dist is not None:
            dist.barrier()
        if has_gpu:
            torch.cuda.synchronize()

    # ---------------------------------------------------------------- per-rank synthetic load
    load = None
    if has_gpu and args.load != "idle":
        from gpumon.ops.load import SyntheticLoad

        load = SyntheticLoad(dev=local_rank, kind=args.load, hbm_bytes=1 << 30).start()
    ar_buf = None
    if dist is not None and args.allreduce_mb > 0:
        # zeros: repeated in-place sums stay finite (ones would reach inf after ~40 steps on 8 ranks)
        ar_buf = torch.zeros(args.allreduce_mb * (1 << 20) // 2, dtype=torch.bfloat16, device=device)

    # ---------------------------------------------------------------- rank 0: exporter + scraper
    mon = None
    core = None
    backend = args.backend
    if rank == 0:
        from gpumon import core as _core
        from gpumon.config import Config
        from gpumon.monitor import GpuMonitor

        core = _core()
        if backend == "auto":
            backend = "amdsmi" if has_gpu else f"mock:gpus={n * args.replicate},mode=load"
            if has_gpu and args.replicate > 1:
                backend = f"amdsmi:replicate={args.replicate}"
        cfg = Config(backend=backend, devices=list(range(n)) if backend.startswith(("amdsmi", "rocm_smi")) else [],
                     interval=args.interval, listen="127.0.0.1:0", http_threads=2, host="bench-node",
                     enable_probe=args.probe and has_gpu, log_level="warn", fast_path=not args.no_fast_path,
                     sample_threads=args.sample_threads)
        mon = GpuMonitor(cfg, control_plane=False).start()
        if mon.start_error:
            raise SystemExit(f"exporter backend failed: {mon.start_error}")
        st = mon.ex.statics()
        if len(st) < n:
            raise SystemExit(f"exporter sees {len(st)} GPU(s), bench needs {n}")
        mon.wait_ticks(args.warmup, timeout_s=args.warmup * args.interval * 5 + 30)

    barrier()
    scrape_result = {}
    scraper = None
    if rank == 0:
        duration = args.steps * args.interval

        def _scrape():
            scrape_result.update(core.scrape_load("127.0.0.1", mon.port, "/metrics", n_requests=0,
                                                  duration_s=duration, concurrency=args.scrape_concurrency,
                                                  rate_hz=args.scrape_rate, keep_alive=True, gzip=args.gzip))

        scraper = threading.Thread(target=_scrape, daemon=True)
        s0 = mon.ex.self_stats()
        seq0 = mon.ex.seq

    if ar_buf is not None:  # RCCL channel/buffer setup stays out of the timed region
        for _ in range(max(1, args.warmup)):
            dist.all_reduce(ar_buf)

    # ---------------------------------------------------------------- timed region
    barrier()
    t0 = time.perf_counter()
    if scraper is not None:
        scraper.start()
    xgmi_rates = []  # per tick: (sum of per-link write B/s, sum of read B/s) per sampled device
    ar_events = []
    for step in range(args.steps):
        if rank == 0:
            if not mon.ex.wait_for_seq(seq0 + step + 1, args.interval * 5 + 10):
                raise SystemExit("exporter tick timed out")
            xgmi_rates.append([(sum(r.get("xgmi_wr_Bps") or [0.0]), sum(r.get("xgmi_rd_Bps") or [0.0]))
                               for r in mon.ex.rates() if r.get("valid")])
        if ar_buf is not None:
            if has_gpu:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
                dist.all_reduce(ar_buf)
                ev[1].record()
                ar_events.append(ev)
            else:
                dist.all_reduce(ar_buf)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # xGMI cross-check (N > 1): RCCL ring all-reduce bus bandwidth vs the exporter's own per-link
    # xGMI counters. A ring all-reduce of S bytes moves 2(n-1)/n * S out of every GPU per call.
    xgmi = None
    if ar_buf is not None:
        nbytes = ar_buf.numel() * ar_buf.element_size()
        ar_ms = [a.elapsed_time(b) for a, b in ar_events] if ar_events else []
        t = torch.tensor([sum(ar_ms) / len(ar_ms) if ar_ms else float("nan")], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ar_mean_s = float(t.item()) * 1e-3
        xgmi = {"allreduce_mb": args.allreduce_mb, "allreduce_ms": round(ar_mean_s * 1e3, 3),
                "allreduce_busbw_GBps": round(2 * (n - 1) / n * nbytes / ar_mean_s / 1e9, 2)
                if ar_mean_s == ar_mean_s and ar_mean_s > 0 else None,
                "expected_tx_GBps_per_gpu": round(2 * (n - 1) / n * nbytes * args.steps / elapsed / 1e9, 3)}

    result = None
    if rank == 0:
        s1 = mon.ex.self_stats()
        if scraper is not None:
            scraper.join(timeout=args.interval * 5 + 30)
        lat = scrape_result.get("latencies_s", [])
        samples = s1["samples"] - s0["samples"]
        ticks = mon.ex.seq - seq0
        tick_mean = (s1["sample_sum_s"] - s0["sample_sum_s"]) / max(1, s1["sample_count"] - s0["sample_count"])
        sm = mon.ex.samples()
        util = [x["fields"].get("gfx_util") for x in sm]
        rows = mon.ex.pod_rows()
        value = samples / elapsed
        lstats = load.stats() if load is not None else {}
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
            "vs_baseline": round(value / max(1, len(sm)) / BASELINE_SAMPLES_PER_GPU, 3),
            "dtype": "bf16",
            "data": ("synthetic" if backend in ("amdsmi", "rocm_smi") else
                     f"synthetic (REHEARSAL: {n} physical GPU(s) each sampled {args.replicate}x)"
                     if backend.startswith("amdsmi:replicate") else "synthetic (mock backend: no GPU visible)"),
            "sampled_devices": len(sm),
            "config": {
                "model": f"gpumon MI355X exporter ({backend.split(':')[0]} backend) + synthetic bf16 MFMA/HBM HIP load",
                "global_batch": n,
                "seq_len": None,
                "parallelism": f"node-local exporter over {n} GPU(s); one rank per GPU"
                               + (", RCCL all-reduce per step" if ar_buf is not None else ""),
                "interval_s": args.interval,
            },
            "scrape_p50_ms": round(_pct(lat, 0.50) * 1e3, 4),
            "scrape_p99_ms": round(_pct(lat, 0.99) * 1e3, 4),
            "scrape_max_ms": round(max(lat) * 1e3, 4) if lat else None,
            "scrapes": len(lat),
            "scrape_errors": scrape_result.get("errors", 0),
            "scrape_body_kb": round(scrape_result.get("bytes", 0) / max(1, len(lat)) / 1024, 2),
            "samples_per_sec_per_gpu": round(value / max(1, len(sm)), 4),
            "ticks": ticks,
            "tick_mean_ms": round(tick_mean * 1e3, 4),
            "tick_p99_ms": round(mon.ex.sample_quantile(0.99) * 1e3, 4),
            "server_scrape_p99_ms": round(mon.ex.scrape_quantile(0.99) * 1e3, 4),
            "overruns": s1["overruns"] - s0["overruns"],
            "backend_call_us": {k: round((v["seconds"] - s0["backend_calls"].get(k, {}).get("seconds", 0.0)) * 1e6
                                         / max(1, v["n"] - s0["backend_calls"].get(k, {}).get("n", 0)), 1)
                                for k, v in s1.get("backend_calls", {}).items()},
            "backend": backend,
            "load": args.load if has_gpu else "none",
            "load_tflops": round(lstats.get("tflops", 0.0), 1) if lstats else None,
            "load_tbps": round(lstats.get("tbps", 0.0), 3) if lstats else None,
            "gfx_util_last": util,
            "procs_seen": len([r for r in rows if not r["idle"]]),
            "proc_rows": [{"pid": r["pid"], "vram_gib": round(r["used_memory_bytes"] / 2 ** 30, 2),
                           "cu_occupancy": r["cu_occupancy"], "gfx_util": r["proc_gfx_util"]}
                          for r in rows if not r["idle"]][:8],
            "xgmi": _xgmi_summary(xgmi, xgmi_rates),
            "reference_samples_per_sec_per_gpu": BASELINE_SAMPLES_PER_GPU,
        }
        mon.stop()
    if load is not None:
        load.stop()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if result is not None:
        line = json.dumps(result)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as fh:
                fh.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
