#!/usr/bin/env python3
"""The exporter next to many GPU processes on one MI355X: K tenant processes (the native HIP
partial-occupancy load, `python -m gpumon load --kind partial`, each its own HIP context, VRAM and
KFD entry) share GPU 0 while an in-process exporter (amdsmi backend, sysfs fast path, 1 Hz)
samples it. Reports per K: tick mean / p99 and its phases, the process rows, `gpu_active_processes`,
occupancy reads per tick, and the exporter threads' CPU -- what per-process attribution costs as
the process count grows (the reference ran one `docker top` per container and one POST per
process row per cycle, /root/reference/gpu.py:174-219).

    python tools/many_tenants.py --counts 1,4,12 --seconds 12 > out.json

K stays <= 14: the gpurun boxes allow 16 GPU processes per command.
"""

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _thread_cpu_s():
    hz = os.sysconf("SC_CLK_TCK")
    tot = 0.0
    for t in os.listdir("/proc/self/task"):
        try:
            s = open(f"/proc/self/task/{t}/stat").read()
        except OSError:
            continue
        if not s[s.index("(") + 1:s.rindex(")")].startswith("gpumon-"):
            continue
        f = s.rsplit(")", 1)[1].split()
        tot += (int(f[11]) + int(f[12])) / hz
    return tot


def run(k, seconds, interval):
    from gpumon import core
    from gpumon.export import promtext

    tenants = [subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "partial", "--duty", "0.3",
                                 "--period", "0.05", "--seconds", str(seconds + 10)], cwd=ROOT,
                                stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True) for _ in range(k)]
    try:
        time.sleep(6)  # HIP contexts up, kernels running
        dead = [t.stderr.read()[-500:] for t in tenants if t.poll() is not None]
        if dead:
            return {"k": k, "error": dead[0]}
        ex = core().Exporter({"backend": "amdsmi", "devices": [0], "serve_http": False, "interval_s": interval,
                              "log_level": "warn"})
        err = ex.start()
        if err:
            return {"k": k, "error": err}
        try:
            ex.wait_for_seq(ex.seq + 3, 30)
            q0, c0, r0 = ex.seq, _thread_cpu_s(), ex.self_stats().get("occupancy_reads", 0)
            t0 = time.time()
            time.sleep(seconds)
            q1, c1, r1 = ex.seq, _thread_cpu_s(), ex.self_stats().get("occupancy_reads", 0)
            wall = time.time() - t0
            ticks = [t for t in ex.tick_log() if q0 < t["seq"] <= q1]
            d = sorted(t["duration_s"] for t in ticks)
            rows = [r for r in ex.pod_rows() if not r["idle"]]
            fam = promtext.parse(ex.metrics_text())
            act = promtext.values(fam, "gpu_active_processes", gpu_id="0")
            return {"k": k, "ticks": len(ticks),
                    "tick_mean_ms": round(sum(d) / len(d) * 1e3, 3) if d else None,
                    "tick_p99_ms": round(d[min(len(d) - 1, int(0.99 * len(d)))] * 1e3, 3) if d else None,
                    "t_device_ms": round(sum(t["t_device"] for t in ticks) / len(ticks) * 1e3, 3) if ticks else None,
                    "t_procs_ms": round(sum(t["t_procs"] for t in ticks) / len(ticks) * 1e3, 3) if ticks else None,
                    "t_attrib_ms": round(sum(t["t_attrib"] for t in ticks) / len(ticks) * 1e3, 3) if ticks else None,
                    "t_render_ms": round(sum(t["t_render"] for t in ticks) / len(ticks) * 1e3, 3) if ticks else None,
                    "process_rows": len(rows), "active_processes": act[0] if act else None,
                    "occupancy_reads_per_tick": round((r1 - r0) / max(1, q1 - q0), 1),
                    "exporter_cpu_millicores": round(1000 * (c1 - c0) / wall, 2),
                    "busy_pct_median": sorted(r["proc_gfx_util"] for r in rows if r["proc_gfx_util"] is not None)[
                        len(rows) // 2] if rows else None}
        finally:
            ex.stop()
    finally:
        for t in tenants:
            t.kill()
        for t in tenants:
            t.wait(30)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--counts", default="1,4,12")
    ap.add_argument("--seconds", type=float, default=12.0)
    ap.add_argument("--interval", type=float, default=1.0)
    a = ap.parse_args()
    out = []
    for k in [int(x) for x in a.counts.split(",")]:
        if k > 14:
            raise SystemExit("at most 14 tenants (16 GPU processes per gpurun command)")
        r = run(k, a.seconds, a.interval)
        print(json.dumps(r), file=sys.stderr, flush=True)
        out.append(r)
    print(json.dumps({"interval_s": a.interval, "runs": out}, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
