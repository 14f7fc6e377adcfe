#!/usr/bin/env python3
"""How often the SMU rewrites gpu_metrics, and what one read costs after a given idle gap (MI355X).

The exporter's device read is a pread of /sys/bus/pci/devices/<bdf>/gpu_metrics on a held fd
(csrc/core/sysfs_fast.cpp). Two questions the bench's capacity run raised (profiles/r3_capacity.md):

  cadence   read back to back for --cadence-s seconds; a new table = a new firmware_timestamp
            (the driver stamps system_clock_counter at every read, so raw bytes always differ):
            distinct tables / s is the refresh rate, the ceiling on fresh samples / s / GPU
  gap       read once every G ms for G in --gaps: p50 / p99 / max read latency per gap (a cold
            read at 1 Hz vs a warm one at kHz rates: SMU fetch or CPU wake-up?)

    python tools/gpu_metrics_cadence.py [--load mixed] > out.json

With --load a `gpumon load` child runs the K2 load meanwhile (the bench's condition).
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import struct
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _metrics_path():
    for p in sorted(glob.glob("/sys/class/drm/card*/device/gpu_metrics")):
        try:
            with open(p, "rb") as fh:
                if len(fh.read()) > 4:
                    return os.path.realpath(p)
        except OSError:
            continue
    raise SystemExit("no readable gpu_metrics file")


def _pct(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, int(q * len(s)))] if s else None


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--cadence-s", type=float, default=2.0)
    ap.add_argument("--gaps", default="0,0.5,2,5,10,20,50,200,1000", help="ms between reads")
    ap.add_argument("--reads", type=int, default=200, help="reads per gap (capped at 12 s per gap)")
    ap.add_argument("--load", default="", help="K2 load kind in a child process (mixed / mfma / hbm)")
    ap.add_argument("--warm-gap", type=float, default=100.0, help="ms of idle before the warm-up variants (0 = off)")
    ap.add_argument("--warm-reads", type=int, default=40)
    args = ap.parse_args()

    path = _metrics_path()
    child = None
    if args.load:
        child = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", args.load, "--seconds", "600"],
                                 cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        time.sleep(5.0)
    out = {"path": path, "load": args.load or "none"}
    try:
        fd = os.open(path, os.O_RDONLY)
        buf = os.pread(fd, 65536, 0)
        out["table_bytes"] = len(buf)
        # cadence: back-to-back reads, distinct firmware tables per second and the gap between
        # rewrites. The driver stamps system_clock_counter (offset 32) at every read, so raw bytes
        # always differ: a new table is a new firmware_timestamp (gpu_metrics v1.8, offset 288).
        fmt, content = buf[2], buf[3]
        out["table_version"] = f"{fmt}.{content}"
        if (fmt, content) != (1, 8):
            raise SystemExit(f"gpu_metrics v{fmt}.{content}: firmware_timestamp offset unknown")

        def stamps(b):
            return struct.unpack_from("<Q", b, 288)[0], struct.unpack_from("<Q", b, 32)[0]

        t_end = time.perf_counter() + args.cadence_s
        fw0, sys0 = stamps(buf)
        last, changes, n, lat = fw0, [], 0, []
        while time.perf_counter() < t_end:
            t0 = time.perf_counter()
            b = os.pread(fd, 65536, 0)
            t1 = time.perf_counter()
            lat.append(t1 - t0)
            n += 1
            fw, sc = stamps(b)
            if fw != last:
                changes.append(t1)
                last = fw
        d = [b - a for a, b in zip(changes, changes[1:])]
        # the firmware timestamp's unit against the driver's ns clock over the whole run
        out["firmware_ts_s_per_driver_s"] = round((fw - fw0) * 1e-8 / max(1e-9, (sc - sys0) * 1e-9), 5)
        out["cadence"] = {"reads": n, "seconds": args.cadence_s, "tables": len(changes),
                          "refresh_hz": round(len(changes) / args.cadence_s, 2),
                          "rewrite_gap_ms_p50": round(_pct(d, 0.5) * 1e3, 3) if d else None,
                          "rewrite_gap_ms_min": round(min(d) * 1e3, 3) if d else None,
                          "rewrite_gap_ms_max": round(max(d) * 1e3, 3) if d else None,
                          "read_us_p50": round(_pct(lat, 0.5) * 1e6, 1), "read_us_p99": round(_pct(lat, 0.99) * 1e6, 1)}
        # gap sweep
        gaps = {}
        for g in [float(x) for x in args.gaps.split(",")]:
            reps = max(5, min(args.reads, int(12000 / max(g, 1e-3))))
            lat = []
            for _ in range(reps):
                if g > 0:
                    time.sleep(g / 1e3)
                t0 = time.perf_counter()
                os.pread(fd, 65536, 0)
                lat.append(time.perf_counter() - t0)
            gaps[str(g)] = {"reads": reps, "p50_us": round(_pct(lat, 0.5) * 1e6, 1),
                            "p99_us": round(_pct(lat, 0.99) * 1e6, 1), "max_us": round(max(lat) * 1e6, 1)}
            print(f"gap {g} ms: {gaps[str(g)]}", file=sys.stderr, flush=True)
        out["gap_sweep"] = gaps
        # After a long gap (--warm-gap ms): is the cold read the CPU's or the SMU's? (a) spin the
        # CPU for 2 ms without touching the device, then read; (b) read once, sleep 3 ms, read again.
        if args.warm_gap > 0:
            warm = {"spin_cpu_2ms": [], "prefetch_3ms": [], "plain": []}
            for _ in range(args.warm_reads):
                for kind, lst in warm.items():
                    time.sleep(args.warm_gap / 1e3)
                    if kind == "spin_cpu_2ms":
                        t_spin = time.perf_counter() + 2e-3
                        while time.perf_counter() < t_spin:
                            pass
                    elif kind == "prefetch_3ms":
                        os.pread(fd, 65536, 0)
                        time.sleep(3e-3)
                    t0 = time.perf_counter()
                    os.pread(fd, 65536, 0)
                    lst.append(time.perf_counter() - t0)
            out["warm_after_gap"] = {"gap_ms": args.warm_gap, **{
                k: {"reads": len(v), "p50_us": round(_pct(v, 0.5) * 1e6, 1), "p90_us": round(_pct(v, 0.9) * 1e6, 1)}
                for k, v in warm.items()}}
            print(f"warm: {out['warm_after_gap']}", file=sys.stderr, flush=True)
        os.close(fd)
    finally:
        if child is not None:
            child.terminate()
            child.wait(timeout=30)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
