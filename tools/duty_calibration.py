#!/usr/bin/env python3
"""Does the exported utilisation track the real GPU duty cycle?

For duty d in {0, 0.25, 0.5, 0.75, 1.0}: run the bf16 MFMA burn with idle gaps so the GPU is busy
a fraction d of wall time (LoadGen measures its own busy time with HIP events), and compare:
  - gpu_gfx_activity_avg_percent   (firmware gfx_activity_acc / accumulation_counter, rates.cpp)
  - gpu_xcd_busy_avg_percent        (per-XCD gfx_busy_acc, mean over the 8 XCDs)
  - node_gpu_gpu_util               (instantaneous average_gfx_activity)
  - PMC GRBM_GUI_ACTIVE %           (rocprofiler-sdk device counting, 0.2 s window)
PMC must be initialised before HIP, so it comes first. Prints one JSON object.
"""

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
    P.init()
    agents = P.agents()
    from gpumon import core as _core
    from gpumon.ops.load import SyntheticLoad

    core = _core()
    ex = core.Exporter({"backend": "amdsmi", "devices": [0], "serve_http": False, "interval_s": 0,
                        "verify_kfd": False})
    assert ex.start() == ""
    rows = []
    for duty in (0.0, 0.25, 0.5, 0.75, 1.0):
        load = SyntheticLoad(0, "mfma", duty=duty if duty > 0 else 1.0, mfma_iters=2048) if duty > 0 else None
        if load:
            load.start()
        time.sleep(1.0)
        ex.tick()
        s0 = load.stats() if load else None
        t0 = time.monotonic()
        acts, xcds, insts = [], [], []
        for _ in range(4):
            time.sleep(0.5)
            ex.tick()
            r = ex.rates()[0]
            sm = ex.samples()[0]
            if r.get("valid"):
                acts.append(r["gfx_activity_avg_pct"])
                xb = r.get("xcd_busy_avg") or []
                if xb:
                    xcds.append(sum(xb) / len(xb))
            insts.append(sm["fields"]["gfx_util"])
        wall = time.monotonic() - t0
        s1 = load.stats() if load else None
        pmc = derive(P.sample(0, DEFAULT_COUNTERS, 0.2), agents[0])
        if load:
            load.stop()
        true_busy = (s1["busy_s"] - s0["busy_s"]) / wall * 100 if load else 0.0
        rows.append({"duty_target": duty, "duty_measured_pct": round(true_busy, 1),
                     "gfx_activity_avg_pct": round(sum(acts) / len(acts), 1) if acts else None,
                     "xcd_busy_avg_pct": round(sum(xcds) / len(xcds), 1) if xcds else None,
                     "gfx_util_inst_mean": round(sum(insts) / len(insts), 1),
                     "pmc_gui_active_pct": round(pmc.get("gui_active", 0.0), 1),
                     "pmc_mfma_busy_pct": round(pmc.get("mfma_busy", 0.0), 1)})
        time.sleep(0.5)
    ex.stop()
    print(json.dumps({"rows": rows}))


if __name__ == "__main__":
    main()
