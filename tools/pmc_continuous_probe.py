#!/usr/bin/env python3
"""Continuous PMC counting on MI355X: read semantics and aliasing vs the windowed sampler.

1. semantics: under a constant MFMA burn (child process), read a running device-counting context
   every 100 ms without stopping it; GRBM_COUNT tells whether a read returns the count since the
   context start (cumulative) or since the previous read (reset-on-read).
2. accuracy: for duty loads (fine-grained 25/50/75 % and 150 ms / 500 ms bursts) compare the
   wall-time MFMA busy % from (a) continuous reads once per second and (b) the windowed sampler
   (0.2 s window per second) against the child's own event-timed busy fraction x the full-load
   MFMA busy %.

    python tools/pmc_continuous_probe.py > out.json      (prints progress to stderr)
"""

from __future__ import annotations

import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

COUNTERS = ["GRBM_COUNT", "GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_BF16"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def child(kind="mfma", duty=1.0, period=0.0, seconds=8.0):
    return subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", kind, "--duty", str(duty),
                             "--period", str(period), "--seconds", str(seconds)], cwd=ROOT,
                            stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)


def vals(d):
    return {c: (d[c]["max"] if c.startswith("GRBM") else d[c]["sum"]) for c in COUNTERS if c in d}


def main() -> int:
    from gpumon import _pmc

    _pmc.init()
    ag = _pmc.agents()[0]
    simds = ag["simd_count"] or ag["cu_count"] * 4
    out = {"agent": ag}

    # ---- 1. semantics
    p = child("mfma", seconds=10)
    time.sleep(4.0)
    reads = []
    t0 = time.perf_counter()
    for _ in range(21):
        r = _pmc.read_running([0], COUNTERS)
        reads.append({"t": time.perf_counter() - t0, "started": r["started"], **vals(r["agents"][0] or {})})
        time.sleep(0.1)
    _pmc.stop_running()
    p.communicate(timeout=60)
    g = [x["GRBM_COUNT"] for x in reads[1:]]
    cumulative = all(b > a for a, b in zip(g, g[1:])) and g[-1] > 5 * g[0]
    out["semantics"] = {"reads": reads, "cumulative": cumulative}
    log("semantics:", "cumulative" if cumulative else "reset-on-read", [round(x / 1e6, 1) for x in g[:6]])

    def interval_values(seq):
        res = []
        for a, b in zip(seq, seq[1:]):
            iv = {c: (b[c] - a[c]) if cumulative else b[c] for c in COUNTERS if c in a and c in b}
            iv["dt"] = b["t"] - a["t"]
            iv["gfx_act"] = b.get("gfx_act")
            iv["gfxclk"] = b.get("gfxclk")
            res.append(iv)
        return res

    # firmware-side view of the same intervals: amdsmi gfx activity accumulator (wall-time busy %)
    # and the average gfx clock, from the exporter ticked at each continuous read
    from gpumon import core as _core

    ex = _core().Exporter({"backend": "amdsmi", "devices": [0], "serve_http": False, "interval_s": 0.0,
                           "processes": False, "ras_every": 0})
    ex_err = ex.start()
    if ex_err:
        log("exporter:", ex_err)

    def fw():
        if ex_err:
            return {}
        ex.tick()
        r = ex.rates()[0]
        f = ex.samples()[0]["fields"]
        return {"gfx_act": r.get("gfx_activity_avg_pct"), "gfxclk": f.get("gfxclk_avg") or f.get("gfxclk_cur")}

    # ---- 2. accuracy per pattern
    patterns = [("full", 1.0, 0.0), ("duty25", 0.25, 0.0), ("duty50", 0.5, 0.0), ("duty75", 0.75, 0.0),
                ("burst150", 0.5, 0.3), ("burst500", 0.5, 1.0), ("burst150_25", 0.25, 0.6)]
    full_busy = None
    out["patterns"] = []
    for name, duty, period in patterns:
        secs = 6.0
        p = child("mfma", duty, period, seconds=secs * 2 + 6)
        time.sleep(3.0)
        # (a) continuous: one read per second
        seq = []
        for _ in range(int(secs) + 1):
            r = _pmc.read_running([0], COUNTERS)
            seq.append({"t": time.perf_counter(), **vals(r["agents"][0] or {}), **fw()})
            time.sleep(1.0)
        _pmc.stop_running()
        cont, raw = [], interval_values(seq)
        for iv in raw:
            if iv.get("GRBM_COUNT"):
                cont.append(100.0 * iv["SQ_VALU_MFMA_BUSY_CYCLES"] / (iv["GRBM_COUNT"] * simds))
        # (b) windowed: 0.2 s window per second (the r1 sampler)
        win = []
        for _ in range(int(secs)):
            t = time.perf_counter()
            r = _pmc.sample_many([0], COUNTERS, 0.2)[0]
            v = vals(r or {})
            if v.get("GRBM_COUNT"):
                win.append(100.0 * v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_COUNT"] * simds))
            time.sleep(max(0.0, 1.0 - (time.perf_counter() - t)))
        so, _ = p.communicate(timeout=120)
        st = json.loads(so.strip().splitlines()[-1])
        busy_frac = st["busy_s"] / st["wall_s"] if st.get("wall_s") else None
        row = {"pattern": name, "duty": duty, "period_s": period, "child_busy_frac": busy_frac,
               "cont_mean": statistics.fmean(cont) if cont else None,
               "cont_sd": statistics.pstdev(cont) if len(cont) > 1 else None, "cont": cont,
               "win_mean": statistics.fmean(win) if win else None,
               "win_sd": statistics.pstdev(win) if len(win) > 1 else None, "win": win, "raw": raw}
        if name == "full":
            full_busy = row["cont_mean"]
        if full_busy and busy_frac is not None:
            row["expected"] = full_busy * busy_frac
        out["patterns"].append(row)
        log(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()
                        if k not in ("cont", "win", "raw")}))
        if raw:
            iv = raw[len(raw) // 2]
            log("   raw:", {k: (round(v / 1e6, 2) if isinstance(v, (int, float)) and v and v > 1e5 else v)
                            for k, v in iv.items()})
    if not ex_err:
        ex.stop()
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
