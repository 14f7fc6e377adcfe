#!/usr/bin/env python3
"""In-kernel resident-wave pressure (K1 probe HW_ID.WAVE_ID) vs rocprofiler device-counting
occupancy, idle and under each K2 load kind. Fresh process: PMC registers before HIP initialises.

For every condition: 8 probe launches (1024 one-wave workgroups each) -> per launch the mean over
SIMDs of the lowest wave slot a probe wave got, the histogram of those minima, and the PMC
occupancy % over a 0.2 s window taken right before. Prints one JSON line (profiles/, GPU test)."""

import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))  # oracles
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))  # oracles


def probe_stats(H, probe, n=8):
    means, xcc, hist, lat = [], [], collections.Counter(), []
    for _ in range(n):
        slot = probe.launch()
        r = probe.poll(slot, 5.0)
        if r is None:
            continue
        means.append(r["wave_slot_mean"])
        xcc.append(r["xcc_wave_slot"][:8])
        lat.append(r["host_latency_s"])
        simd_min = {}
        for (x, hw, *_rest) in r["records"]:
            key = (x, (hw >> 8) & 0xFF, (hw >> 4) & 3)
            simd_min[key] = min(simd_min.get(key, 99), hw & 0xF)
        hist.update(simd_min.values())
    return {"wave_slot_mean": sum(means) / max(1, len(means)), "per_launch": means,
            "xcc_mean": [sum(c) / len(xcc) for c in zip(*xcc)] if xcc else [],
            "min_slot_hist": dict(sorted(hist.items())), "latency_ms": [round(v * 1e3, 3) for v in lat]}


def main():
    from oracles.ops.pmc import derive, pmc_module

    # per-wave SQ_WAVE_CYCLES: valid here because the loads run in THIS process
    # (profiles/r1_pmc_cross_process.md)
    occ = ["SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]

    P = pmc_module()
    P.init()
    agent = P.agents()[0]
    from gpumon import hip
    from gpumon.ops.load import SyntheticLoad

    H = hip()
    probe = H.Probe(0, 1024, 4, 200)
    out = {"max_waves_per_cu": agent["max_waves_per_cu"], "simd_count": agent["simd_count"]}
    out["idle"] = probe_stats(H, probe)
    out["idle"]["pmc"] = derive(P.sample(0, occ, 0.2), agent)
    for kind in ("mfma", "hbm", "partial"):
        with SyntheticLoad(0, kind):
            time.sleep(1.0)
            pmc = derive(P.sample(0, occ, 0.2), agent)
            out[kind] = probe_stats(H, probe)
            out[kind]["pmc"] = pmc
    print(json.dumps(out))


if __name__ == "__main__":
    main()
