#!/usr/bin/env python3
"""Tick cadence on a CPU-saturated node, with and without rt_priority (SCHED_FIFO sampler + device
workers). Starts --hogs busy-loop processes (2 per CPU by default), then runs the exporter at
--interval with rt_priority 0 and N in alternating windows, and reports from the tick log how late
ticks started after their deadline (t_late) and how long they took (duration).

    python tools/rt_contention.py --backend mock:gpus=8 --seconds 10 > out.json
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _q(xs, p):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(p * (len(xs) - 1)))] if xs else float("nan")


def window(core, backend, interval, seconds, prio):
    ex = core.Exporter({"backend": backend, "serve_http": False, "interval_s": interval, "rt_priority": prio,
                        "log_level": "error"})
    assert ex.start() == ""
    try:
        time.sleep(seconds)
        rt = ex.self_stats().get("rt_threads", 0)
        log = ex.tick_log()[1:]
    finally:
        ex.stop()
    late = [t["t_late"] * 1e3 for t in log]
    dur = [t["duration_s"] * 1e3 for t in log]
    return {"rt_priority": prio, "rt_threads": rt, "ticks": len(log),
            "late_ms_p50": round(_q(late, 0.5), 3), "late_ms_p99": round(_q(late, 0.99), 3),
            "late_ms_max": round(max(late), 3) if late else None,
            "tick_ms_p50": round(_q(dur, 0.5), 3), "tick_ms_p99": round(_q(dur, 0.99), 3),
            "tick_ms_max": round(max(dur), 3) if dur else None}


def main() -> int:
    from gpumon import core as _core

    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="mock:gpus=8")
    ap.add_argument("--interval", type=float, default=0.1)
    ap.add_argument("--seconds", type=float, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--prio", type=int, default=10)
    ap.add_argument("--hogs", type=int, default=2 * (os.cpu_count() or 4))
    a = ap.parse_args()
    core = _core()
    hogs = [subprocess.Popen([sys.executable, "-c", "while True: pass"]) for _ in range(a.hogs)]
    out = {"backend": a.backend, "interval_s": a.interval, "hogs": a.hogs, "cpus": os.cpu_count(), "windows": []}
    try:
        time.sleep(1)
        for _ in range(a.rounds):
            for prio in (0, a.prio):
                w = window(core, a.backend, a.interval, a.seconds, prio)
                out["windows"].append(w)
                print(w, file=sys.stderr, flush=True)
    finally:
        for h in hogs:
            h.kill()
        for h in hogs:
            h.wait()
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
