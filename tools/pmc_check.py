#!/usr/bin/env python3
"""PMC validation in a fresh process (rocprofiler must register before HSA init):
idle vs bf16-MFMA burn vs HBM stream, device-wide MFMA-busy / occupancy via device counting.
Prints one JSON line. Used by tests/test_gpu_pmc.py and for profiles/."""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))  # oracles
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))  # oracles


def main():
    from oracles.ops.pmc import DEFAULT_COUNTERS, derive, pmc_module

    P = pmc_module()
    n = P.init()
    agents = P.agents()
    out = {"agents": agents, "n": n}
    counters = DEFAULT_COUNTERS
    # occupancy needs the per-wave SQ_WAVE_CYCLES, which counts only this process's waves: valid
    # here because SyntheticLoad runs in-process (the exporter's default set leaves it out)
    occ = ["SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]

    def measure():
        d = derive(P.sample(0, counters, 0.2), agents[0], 0.2)
        d["occupancy"] = derive(P.sample(0, occ, 0.2), agents[0]).get("occupancy", 0.0)
        return d

    raw = P.sample(0, counters, 0.2)
    out["idle"] = measure()
    out["idle_raw"] = raw
    from gpumon.ops.load import SyntheticLoad

    for kind in ("mfma", "hbm", "partial"):
        with SyntheticLoad(0, kind) as load:
            time.sleep(1.0)
            raw = P.sample(0, counters, 0.2)
            out[kind] = measure()
            out[kind + "_raw"] = {k: {"sum": v["sum"], "max": v["max"], "n": v["n"]} for k, v in raw.items()}
            out[kind + "_load"] = load.stats()
            if kind == "mfma":  # shared-window path used by PmcRunner on multi-GPU nodes
                many = P.sample_many(list(range(len(agents))), counters, 0.2)
                out["mfma_many"] = [derive(r, agents[i], 0.2) if r is not None else None for i, r in enumerate(many)]
    print(json.dumps(out, default=str))


if __name__ == "__main__":
    main()
