#!/usr/bin/env python3
"""Can the PMC owner be frozen between reads? (MI355X experiment)

rocprofiler-sdk's device counting service leaves an HSA async-events thread polling (ioctl +
calloc in a loop: one full core, profiles/r2_footprint.md). This drives a child process that owns
the counting contexts (gpumon._pmc read_running) over a pipe and SIGSTOPs it between reads:
  * CPU of the child while stopped (should be ~0),
  * whether the hardware kept counting across the stop (MFMA busy over a stopped interval must
    match the unstopped one under a constant burn in another process).

    python tools/pmc_stop_probe.py > out.json
"""

from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HZ = os.sysconf("SC_CLK_TCK")
CHILD = r"""
import json, sys
sys.path.insert(0, %r)
from gpumon import _pmc
_pmc.init()
ag = _pmc.agents()[0]
C = ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"]
print(json.dumps({"simds": ag["simd_count"] or ag["cu_count"] * 4}), flush=True)
for line in sys.stdin:
    r = _pmc.read_running([0], C)
    a = r["agents"][0] or {}
    print(json.dumps({k: (a[k]["max"] if k.startswith("GRBM") else a[k]["sum"]) for k in C if k in a}), flush=True)
""" % ROOT


def cpu(pid):
    f = open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()
    return (int(f[11]) + int(f[12])) / HZ


def main() -> int:
    load = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mfma", "--seconds", "40"], cwd=ROOT,
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    ch = subprocess.Popen([sys.executable, "-c", CHILD], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    simds = json.loads(ch.stdout.readline())["simds"]
    time.sleep(4)

    def read():
        ch.stdin.write("r\n")
        ch.stdin.flush()
        return json.loads(ch.stdout.readline()), time.perf_counter()

    out = {"running": [], "stopped": []}
    prev, tp = read()
    for mode in ("running", "stopped", "running", "stopped"):
        c0, t0 = cpu(ch.pid), time.perf_counter()
        if mode == "stopped":
            os.kill(ch.pid, signal.SIGSTOP)
        time.sleep(3.0)
        c1 = cpu(ch.pid)
        if mode == "stopped":
            os.kill(ch.pid, signal.SIGCONT)
        cur, tc = read()
        d = {k: cur[k] - prev[k] for k in cur}
        out[mode].append({"cpu_pct": round(100 * (c1 - c0) / (time.perf_counter() - t0), 2),
                          "interval_s": round(tc - tp, 3),
                          "mfma_busy_active_pct": round(100 * d["SQ_VALU_MFMA_BUSY_CYCLES"]
                                                        / (d["GRBM_GUI_ACTIVE"] * simds), 2),
                          "grbm_count_per_s": round(d["GRBM_COUNT"] / (tc - tp) / 1e9, 3)})
        print(mode, out[mode][-1], file=sys.stderr, flush=True)
        prev, tp = cur, tc
    ch.stdin.close()
    ch.wait(30)
    load.wait(60)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
