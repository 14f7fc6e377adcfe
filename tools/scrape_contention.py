#!/usr/bin/env python3
"""Scrape latency on a CPU-saturated node: the bench's scrape load (200 req/s,
2 keep-alive connections) against an 8-GPU mock exporter at 1 Hz and 10 Hz, with 2 busy loops per
CPU, the HTTP loops at normal priority vs SCHED_FIFO (http_rt_priority, each loop capped at
http_rt_budget of a CPU per 100 ms). The measuring client runs SCHED_FIFO itself (priority 50),
so its own wake-ups do not count against the server; without CAP_SYS_NICE it runs normal and
says so. A last phase floods the RT loops (no rate limit, 8 connections) and reports the CPU
they took and how often they were demoted: the budget, not the request rate, bounds them.

    python tools/scrape_contention.py [--seconds 10] [--rounds 2] > profiles/data/r4_scrape_contention.json
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
    if not xs:
        return None
    k = (len(xs) - 1) * p
    f = int(k)
    c = min(f + 1, len(xs) - 1)
    return xs[f] + (xs[c] - xs[f]) * (k - f)


def _ms(x):
    return round(x * 1e3, 4) if x is not None else None


def _http_cpu_s():
    """CPU seconds of this process's gpumon-http threads (schedstat, ns)."""
    tot = 0.0
    for t in os.listdir("/proc/self/task"):
        try:
            if open(f"/proc/self/task/{t}/comm").read().strip() != "gpumon-http":
                continue
            tot += int(open(f"/proc/self/task/{t}/schedstat").read().split()[0]) * 1e-9
        except (OSError, ValueError, IndexError):
            pass
    return tot


def _client_fifo(on: bool) -> bool:
    try:
        os.sched_setscheduler(0, os.SCHED_FIFO if on else os.SCHED_OTHER, os.sched_param(50 if on else 0))
        return True
    except (PermissionError, OSError):
        return False


def window(core, backend, interval, seconds, http_prio, rate, conc, budget):
    ex = core.Exporter({"backend": backend, "listen_addr": "127.0.0.1", "port": 0, "interval_s": interval,
                        "http_threads": 2, "host": "node", "http_rt_priority": http_prio,
                        "http_rt_budget": budget, "log_level": "error"})
    assert ex.start() == ""
    try:
        ex.wait_for_seq(2, 30)
        n0 = ex.scrape_count()
        cpu0 = _http_cpu_s()
        fifo = _client_fifo(True)  # threads the client starts now inherit it
        try:
            r = core.scrape_load("127.0.0.1", ex.port, "/metrics", n_requests=0, duration_s=seconds,
                                 concurrency=conc, rate_hz=rate, keep_alive=True, gzip=False)
        finally:
            _client_fifo(False)
        cpu1 = _http_cpu_s()
        lat = r.get("latencies_s", [])
        deadline = time.time() + 2
        while ex.scrape_count() - n0 < len(lat) and time.time() < deadline:
            time.sleep(0.01)
        srv = list(ex.scrape_durations_since(n0))
        st = ex.self_stats()
    finally:
        ex.stop()
    return {"interval_s": interval, "http_rt_priority": http_prio, "client_fifo": fifo, "rate_hz": rate,
            "connections": conc, "scrapes": len(lat), "errors": r.get("errors", 0),
            "body_kb": round(r.get("bytes", 0) / max(1, len(lat)) / 1024, 1),
            "client_p50_ms": _ms(_q(lat, 0.5)), "client_p99_ms": _ms(_q(lat, 0.99)),
            "client_p999_ms": _ms(_q(lat, 0.999)), "client_max_ms": _ms(max(lat) if lat else None),
            "server_p99_ms": _ms(_q(srv, 0.99)), "server_p999_ms": _ms(_q(srv, 0.999)),
            "http_cpu_share": round((cpu1 - cpu0) / seconds, 4),
            "http_rt_loops": st.get("http_rt_loops"), "http_rt_demotions": st.get("http_rt_demotions")}


def main() -> int:
    from gpumon import core as _core

    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="mock:gpus=8,mode=load")
    ap.add_argument("--intervals", default="1.0,0.1")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--rate", type=float, default=200.0)
    ap.add_argument("--prio", type=int, default=10)
    ap.add_argument("--budget", type=float, default=0.2)
    ap.add_argument("--hogs", type=int, default=2 * (os.cpu_count() or 4))
    ap.add_argument("--spinners", type=int, default=os.cpu_count() or 4,
                    help="SCHED_IDLE spinners of the idle-state check (the box's CPU share, not the machine's)")
    ap.add_argument("--flood-s", type=float, default=5.0)
    a = ap.parse_args()
    core = _core()
    out = {"backend": a.backend, "cpus": os.cpu_count(), "hogs": a.hogs, "seconds": a.seconds, "windows": []}
    # quiet reference first (normal and RT loops), then the same with SCHED_IDLE spinners on every
    # CPU: they take no CPU from anything runnable but keep the CPUs out of their idle states, so
    # any difference is the cost of waking an idle CPU (C-state exit / a halted vCPU), not
    # contention. Then the same windows under real (SCHED_OTHER) hogs.
    ivs = [float(x) for x in a.intervals.split(",")]
    for _ in range(a.rounds):
        for iv in ivs:
            for prio in (0, a.prio):
                out["windows"].append(dict(window(core, a.backend, iv, a.seconds, prio, a.rate, 2, a.budget),
                                           hogs=0))
    idle_code = "import os; os.sched_setscheduler(0, os.SCHED_IDLE, os.sched_param(0))\nwhile True: pass"
    spin = [subprocess.Popen([sys.executable, "-c", idle_code]) for _ in range(a.spinners)]
    try:
        time.sleep(1.0)
        for _ in range(a.rounds):
            for iv in ivs:
                out["windows"].append(dict(window(core, a.backend, iv, a.seconds, 0, a.rate, 2, a.budget),
                                           hogs=0, idle_spinners=len(spin)))
    finally:
        for h in spin:
            h.kill()
        for h in spin:
            h.wait()
    hogs = [subprocess.Popen([sys.executable, "-c", "while True: pass"]) for _ in range(a.hogs)]
    try:
        time.sleep(1.0)
        for _ in range(a.rounds):
            for iv in ivs:
                for prio in (0, a.prio):  # alternating A/B windows
                    out["windows"].append(dict(window(core, a.backend, iv, a.seconds, prio, a.rate, 2, a.budget),
                                               hogs=a.hogs))
        # flood: unthrottled, 8 connections, RT loops -- how much CPU do they take?
        fl = window(core, a.backend, 1.0, a.flood_s, a.prio, 0.0, 8, a.budget)
        fl["note"] = "flood: no rate limit, 8 connections; http_cpu_share is CPU-seconds per second over 2 loops"
        out["flood"] = fl
    finally:
        for h in hogs:
            h.kill()
        for h in hogs:
            h.wait()
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
