#!/usr/bin/env python3
"""Per-operand-type MFMA burns vs the PMC MOPS counters (gpu_mfma_tflops{dtype}) on one MI355X.

For each matrix path (bf16, f16, fp8, f32, f64, i8, and the block-scaled f8f6f4 path with fp8 and
fp4 operands): the K2 load generator burns that path (its FLOPs timed with HIP events) while a
0.4 s device-counting window samples every MOPS counter. Prints one JSON line: per dtype the
event-timed TFLOP/s, the TFLOP/s each MOPS counter reported, and MFMA busy. Fresh process, no torch
(PMC registers before HIP; a second HIP runtime in the process would trip the profiler)."""
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
    agent = P.agents()[0]
    from gpumon.ops.load import SyntheticLoad

    res = {}
    for dt in sys.argv[1:] or ("bf16", "f16", "fp8", "mxfp8", "mxfp4", "i8", "f32", "f64"):
        # long launches (7-30 ms): the host sync between 4-launch batches stays < 0.5 % of the window
        with SyntheticLoad(0, "mfma", mfma_dtype=dt, mfma_iters=16384) as load:
            time.sleep(1.0)
            s0 = load.stats()
            raw = P.sample(0, DEFAULT_COUNTERS, 0.4)
            time.sleep(0.6)
            s1 = load.stats()
        d = derive(raw, agent, 0.4)
        ev = (s1["flops"] - s0["flops"]) / max(1e-9, s1["mfma_s"] - s0["mfma_s"]) / 1e12
        res[dt] = {"event_tflops": round(ev, 1),
                   "pmc_tflops": {k: round(v, 1) for k, v in d.get("mfma_tflops", {}).items() if v > 0.05},
                   "mfma_busy": round(d.get("mfma_busy", 0.0), 1)}
        print(dt, res[dt], file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
