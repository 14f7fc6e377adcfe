#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) into a markdown table.

    python tools/prof_summary.py gpurun_out/round/prof/bench_results.db > profiles/x.md

Columns: kernel, calls, total ms, mean us, share, grid, workgroup, VGPR/AGPR/SGPR, LDS.
Optional --flops / --bytes per-kernel annotations turn the mean time into TFLOP/s or TB/s.
"""

import argparse
import sqlite3
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--flops", action="append", default=[], help="substring=FLOP_per_call")
    ap.add_argument("--bytes", action="append", default=[], help="substring=bytes_per_call")
    a = ap.parse_args()
    flops = {k: float(v) for k, v in (x.split("=", 1) for x in a.flops)}
    nbytes = {k: float(v) for k, v in (x.split("=", 1) for x in a.bytes)}
    c = sqlite3.connect(a.db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration), "
        "max(grid_x), max(workgroup_x), max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), "
        "max(lds_size) from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = sys.stdout
    out.write("| kernel | calls | total ms | mean us | min us | max us | share | grid | wg | vgpr/agpr/sgpr | lds | rate |\n")
    out.write("|---|---|---|---|---|---|---|---|---|---|---|---|\n")
    for (name, n, tot, avg, mn, mx, gx, wx, v, ag, s, lds) in rows:
        # rocpd durations are in ns
        rate = ""
        for k, f in flops.items():
            if k in name:
                rate = f"{f / (avg * 1e-9) / 1e12:.0f} TFLOP/s"
        for k, b in nbytes.items():
            if k in name:
                rate = f"{b / (avg * 1e-9) / 1e12:.2f} TB/s"
        short = name if len(name) < 70 else name[:67] + "..."
        out.write(f"| `{short}` | {n} | {tot / 1e6:.2f} | {avg / 1e3:.1f} | {mn / 1e3:.1f} | {mx / 1e3:.1f} | "
                  f"{100.0 * tot / total:.1f}% | {gx} | {wx} | {v}/{ag}/{s} | {lds} | {rate} |\n")


if __name__ == "__main__":
    main()
