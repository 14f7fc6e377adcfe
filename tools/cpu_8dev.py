#!/usr/bin/env python3
"""Exporter CPU at 10 Hz with 1 and 8 devices, split by thread (profiles/r5_cpu_8dev.md).

Each shape starts `bin/gpumon-exporter` at --interval 0.1 and scrapes /metrics 10 times a second with
`Accept-Encoding: gzip` over one keep-alive connection (Prometheus' shape), then reads every thread's
utime+stime from /proc over the window. Shapes:

  mock1 / mock8          the mock backend with 1 / 8 GPUs (no device I/O: the exporter's own cost)
  amdsmi1 / amdsmi8      the real backend, the one GPU sampled 1x / 8x (amdsmi:replicate=8)
  amdsmi8_seq            the same with sample_threads=0: no per-GPU workers, one thread reads all 8

The amdsmi shapes run next to the mixed K2 load (the stress configuration). `--only mock1,mock8`
runs a subset (the mock shapes run without a GPU).

    python tools/cpu_8dev.py --seconds 20 --out gpurun_out/r5/cpu8.jsonl
"""

from __future__ import annotations

import argparse
import http.client
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from thread_cpu import threads  # noqa: E402

SHAPES = {  # name: (flags, extra environment)
    "mock1": (["--backend", "mock:gpus=1"], {}),
    "mock8": (["--backend", "mock:gpus=8"], {}),
    "amdsmi1": (["--backend", "amdsmi"], {}),
    "amdsmi8": (["--backend", "amdsmi:replicate=8"], {}),
    "amdsmi8_seq": (["--backend", "amdsmi:replicate=8", "--sample-threads", "0"], {}),
    # which per-device work contends when 8 workers read ONE physical GPU (the rehearsal's shape)
    "amdsmi8_occ1": (["--backend", "amdsmi:replicate=8"], {"GPUMON_OCC_SAMPLES": "1"}),
    "amdsmi8_noprewarm": (["--backend", "amdsmi:replicate=8", "--prewarm-ms", "0"], {}),
    "amdsmi1_occ1": (["--backend", "amdsmi"], {"GPUMON_OCC_SAMPLES": "1"}),
}
DEFAULT = ["mock1", "mock8", "amdsmi1", "amdsmi8", "amdsmi8_seq"]


def thread_times(pid):
    """tid -> (name, utime s, stime s): user space vs kernel (a contended driver lock spins in stime)."""
    out = {}
    hz = os.sysconf("SC_CLK_TCK")
    for t in os.listdir(f"/proc/{pid}/task"):
        try:
            with open(f"/proc/{pid}/task/{t}/stat") as fh:
                s = fh.read()
            f = s.rsplit(")", 1)[1].split()
            out[int(t)] = (s[s.index("(") + 1:s.rindex(")")], int(f[11]) / hz, int(f[12]) / hz)
        except (OSError, ValueError):
            pass
    return out


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def scraper(port, hz, stop, stats):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    period, nxt = 1.0 / hz, time.monotonic()
    while not stop.is_set():
        nxt += period
        try:
            c.request("GET", "/metrics", headers={"Accept-Encoding": "gzip"})
            r = c.getresponse()
            body = r.read()
            stats["n"] += 1
            stats["bytes"] = len(body)
        except (OSError, http.client.HTTPException):
            stats["err"] += 1
            c.close()
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
        d = nxt - time.monotonic()
        if d > 0:
            stop.wait(d)


def sample_hist(port):
    """(sum, count) of gpumon_sample_duration_seconds: the tick's own time (sample + render + publish)."""
    try:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
        c.request("GET", "/metrics")
        text = c.getresponse().read().decode()
    except (OSError, http.client.HTTPException):
        return None
    vals = {}
    for line in text.splitlines():
        for k in ("_sum", "_count"):
            if line.startswith("gpumon_sample_duration_seconds" + k):
                vals[k] = float(line.rsplit(" ", 1)[1])
    return (vals["_sum"], vals["_count"]) if len(vals) == 2 else None


def measure(name, shape, seconds, scrape_hz):
    flags, env = shape
    port = free_port()
    ex = subprocess.Popen([os.path.join(ROOT, "bin", "gpumon-exporter"), "--interval", "0.1", "--listen",
                           f"127.0.0.1:{port}", "--log-level", "warn", "--no-pod-resources", "--no-cri", *flags],
                          stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=dict(os.environ, **env))
    stop, stats = threading.Event(), {"n": 0, "err": 0, "bytes": 0}
    th = None
    try:
        time.sleep(4)
        if ex.poll() is not None:
            raise SystemExit(f"{name}: exporter exited: {ex.stderr.read()[-2000:]}")
        th = threading.Thread(target=scraper, args=(port, scrape_hz, stop, stats), daemon=True)
        th.start()
        time.sleep(3)
        h0 = sample_hist(port)
        t0, a0, s0, u0 = time.time(), threads(ex.pid), dict(stats), thread_times(ex.pid)
        time.sleep(seconds)
        t1, a1, s1, u1 = time.time(), threads(ex.pid), dict(stats), thread_times(ex.pid)
        h1 = sample_hist(port)
        dt = t1 - t0
        by_name = {}
        for tid, (tname, c1, _) in a1.items():
            c0 = a0.get(tid, (tname, 0.0, ""))[1]
            by_name.setdefault(tname, []).append(round(1000 * (c1 - c0) / dt, 2))
        total = sum(sum(v) for v in by_name.values())
        user = sum(u1[t][1] - u0.get(t, ("", 0.0, 0.0))[1] for t in u1)
        sys_ = sum(u1[t][2] - u0.get(t, ("", 0.0, 0.0))[2] for t in u1)
        tick = None
        if h0 and h1 and h1[1] > h0[1]:
            tick = {"mean_ms": round(1000 * (h1[0] - h0[0]) / (h1[1] - h0[1]), 3), "ticks": int(h1[1] - h0[1])}
        return {"shape": name, "flags": flags, "seconds": round(dt, 2), "scrape_hz": scrape_hz,
                "scrapes": s1["n"] - s0["n"], "scrape_errors": s1["err"] - s0["err"], "body_bytes_gzip": s1["bytes"],
                "total_millicores": round(total, 1), "env": env,
                "user_millicores": round(1000 * user / dt, 1), "sys_millicores": round(1000 * sys_ / dt, 1),
                "threads_millicores": {k: sorted(v, reverse=True) for k, v in sorted(by_name.items(), key=lambda kv: -sum(kv[1]))},
                "tick": tick}
    finally:
        stop.set()
        if th is not None:
            th.join(10)
        ex.terminate()
        try:
            ex.wait(20)
        except subprocess.TimeoutExpired:
            ex.kill()
            ex.wait()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20)
    ap.add_argument("--scrape-hz", type=float, default=10)
    ap.add_argument("--only", default="", help="comma-separated shapes (default all)")
    ap.add_argument("--no-load", action="store_true", help="no K2 load next to the amdsmi shapes")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    names = [s for s in (a.only.split(",") if a.only else DEFAULT) if s]
    load = None
    if any(n.startswith("amdsmi") for n in names) and not a.no_load:
        total = len(names) * (a.seconds + 12) + 30
        load = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mixed", "--seconds", str(total)],
                                cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        time.sleep(5)
    try:
        for n in names:
            row = measure(n, SHAPES[n], a.seconds, a.scrape_hz)
            row["loaded"] = load is not None and n.startswith("amdsmi")
            line = json.dumps(row)
            print(line, flush=True)
            if a.out:
                with open(a.out, "a") as fh:
                    fh.write(line + "\n")
    finally:
        if load is not None:
            load.terminate()
            load.wait(60)
    return 0


if __name__ == "__main__":
    sys.exit(main())
