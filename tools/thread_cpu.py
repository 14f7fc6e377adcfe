#!/usr/bin/env python3
"""Per-thread CPU of an exporter configuration (which thread spends the footprint?).

Starts `bin/gpumon-exporter <flags>` next to a mixed K2 load process, lets it settle, then reports
each thread's name and CPU share over a measurement window from /proc/<pid>/task/*/stat.

    python tools/thread_cpu.py --seconds 15 -- --interval 0.1 --pmc
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HZ = os.sysconf("SC_CLK_TCK")


def threads(pid):
    out = {}
    for t in os.listdir(f"/proc/{pid}/task"):
        try:
            with open(f"/proc/{pid}/task/{t}/stat") as fh:
                s = fh.read()
            name = s[s.index("(") + 1:s.rindex(")")]
            f = s.rsplit(")", 1)[1].split()
            out[int(t)] = (name, (int(f[11]) + int(f[12])) / HZ, f[0])
        except (OSError, ValueError):
            pass
    return out


def rss_mb(pid):
    with open(f"/proc/{pid}/status") as fh:
        for line in fh:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024
    return None


def rss_by_mapping(pid, top=8):
    """RSS (MB) aggregated by mapped file / anonymous, largest first (from /proc/<pid>/smaps)."""
    agg, cur = {}, None
    with open(f"/proc/{pid}/smaps") as fh:
        for line in fh:
            parts = line.split()
            if not parts:
                continue
            if "-" in parts[0] and len(parts) >= 5 and not parts[0].endswith(":"):
                cur = parts[5] if len(parts) >= 6 else "[anon]"
            elif parts[0] == "Rss:" and cur is not None:
                agg[cur] = agg.get(cur, 0) + int(parts[1])
    return [(k, round(v / 1024, 1)) for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:top]]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=15)
    ap.add_argument("--no-load", action="store_true")
    ap.add_argument("--env", action="append", default=[], help="K=V for the exporter process")
    ap.add_argument("flags", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    flags = [f for f in a.flags if f != "--"]
    load = None
    if not a.no_load:
        load = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mixed", "--seconds",
                                 str(a.seconds + 30)], cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        time.sleep(5)
    ex = subprocess.Popen([os.path.join(ROOT, "bin", "gpumon-exporter"), "--backend", "amdsmi", "--listen",
                           "127.0.0.1:0", "--log-level", "warn", "--no-pod-resources", "--no-cri", *flags],
                          stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                          env=dict(os.environ, **dict(kv.split("=", 1) for kv in a.env)))
    try:
        time.sleep(8)
        if ex.poll() is not None:
            raise SystemExit(ex.stderr.read()[-2000:])
        def kids():
            out = []
            for p in os.listdir("/proc"):  # the PMC helper (ondevice_isolate): its CPU counts for the pod too
                if p.isdigit():
                    try:
                        if int(open(f"/proc/{p}/stat").read().rsplit(")", 1)[1].split()[1]) == ex.pid:
                            out.append(int(p))
                    except (OSError, ValueError, IndexError):
                        pass
            return out

        def kid_cpu(k):
            return sum(v[1] for v in threads(k).values())

        k0 = {k: kid_cpu(k) for k in kids()}
        t0, a0 = time.time(), threads(ex.pid)
        time.sleep(a.seconds)
        t1, a1 = time.time(), threads(ex.pid)
        dt = t1 - t0
        rows = []
        for tid, (name, c1, state) in a1.items():
            c0 = a0.get(tid, (name, 0.0, ""))[1]
            row = {"tid": tid, "name": name, "cpu_pct": round(100 * (c1 - c0) / dt, 2), "state": state}
            for f in ("wchan", "syscall"):
                try:
                    with open(f"/proc/{ex.pid}/task/{tid}/{f}") as fh:
                        row[f] = fh.read().strip()[:60]
                except OSError as e:
                    row[f] = f"ERR{e.errno}"
            rows.append(row)
        rows.sort(key=lambda r: -r["cpu_pct"])
        # the hottest thread: is it spinning in user space or polling a syscall?
        if rows and rows[0]["cpu_pct"] > 20:
            tid = rows[0]["tid"]
            base = f"/proc/{ex.pid}/task/{tid}"

            def kv(path):
                d = {}
                try:
                    for line in open(path):
                        k, _, v = line.partition(":")
                        d[k.strip()] = v.strip()
                except OSError:
                    pass
                return d

            io0, st0 = kv(base + "/io"), kv(base + "/status")
            hist = {}
            t_end = time.time() + 1.0
            while time.time() < t_end:
                try:
                    sc = open(base + "/syscall").read().split()[0]
                except (OSError, IndexError):
                    sc = "?"
                hist[sc] = hist.get(sc, 0) + 1
            io1, st1 = kv(base + "/io"), kv(base + "/status")
            rows[0]["syscall_hist"] = dict(sorted(hist.items(), key=lambda x: -x[1])[:6])
            ips = os.path.join(ROOT, "tools", "ip_sample")
            if os.path.exists(ips):  # where in user space it spins (perf_event CPU-clock samples)
                r = subprocess.run([ips, str(ex.pid), str(tid), "1.0"], capture_output=True, text=True, timeout=30)
                try:
                    top = json.loads(r.stdout)["top"]
                    sym = "/opt/rocm/lib/llvm/bin/llvm-symbolizer"
                    for t in top[:6]:
                        if t["map"].startswith("/") and os.path.exists(sym):
                            s = subprocess.run([sym, "--obj=" + t["map"], t["file_off"]], capture_output=True,
                                               text=True, timeout=30)
                            t["sym"] = s.stdout.strip().splitlines()[0][:120] if s.stdout.strip() else ""
                    rows[0]["ip_top"] = top[:6]
                except (ValueError, KeyError):
                    rows[0]["ip_sample_error"] = (r.stderr or r.stdout)[-300:]
            for k in ("syscr", "syscw"):
                if k in io0 and k in io1:
                    rows[0][k + "_per_s"] = int(io1[k]) - int(io0[k])
            for k in ("voluntary_ctxt_switches", "nonvoluntary_ctxt_switches"):
                if k in st0 and k in st1:
                    rows[0][k + "_per_s"] = int(st1[k]) - int(st0[k])
        child_rows = [{"pid": k, "rss_mb": rss_mb(k), "state": open(f"/proc/{k}/stat").read().rsplit(")", 1)[1].split()[0],
                       "cpu_pct": round(100 * (kid_cpu(k) - c0k) / dt, 2)} for k, c0k in k0.items()]
        print(json.dumps({"flags": flags, "env": a.env, "threads": len(rows), "children": child_rows, "rss_mb": rss_mb(ex.pid),
                          "rss_by_mapping": rss_by_mapping(ex.pid),
                          "total_cpu_pct": round(sum(r["cpu_pct"] for r in rows), 2), "top": rows[:8]}), flush=True)
    finally:
        ex.terminate()
        try:
            ex.wait(20)
        except subprocess.TimeoutExpired:
            ex.kill()
        if load is not None:
            load.terminate()
            load.wait(60)
    return 0


if __name__ == "__main__":
    sys.exit(main())
