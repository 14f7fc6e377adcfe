#!/usr/bin/env python3
"""Which device-counting PMCs see waves of OTHER processes? (an exporter never owns the workload)

Per-wave SQ counters (SQ_WAVES, SQ_WAVE_CYCLES, SQ_INSTS_*) are gated by the dispatch's
perf-count enable, which the profiler sets only for its own process's queues; per-SIMD / SPI /
GRBM counters are not. This scans every supported SQ_/SPI_/GRBM_/CPC_/CPF_ base counter, one per
counting window, idle and while a bf16 MFMA burn runs in another process, and prints one JSON line:
{counter: [idle_sum, loaded_sum]}."""
import json
import os
import re
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))  # oracles
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))  # oracles


def scan(P, names, window):
    out = {}
    for n in names:
        try:
            r = P.sample(0, [n], window)
            out[n] = r.get(n, {}).get("sum", None)
        except Exception as e:  # noqa: BLE001
            out[n] = "ERR " + str(e)[:60]
    return out


def main():
    from oracles.ops.pmc import pmc_module

    P = pmc_module()
    P.init()
    names = [n for n in P.supported_counters(0) if re.match(r"^(SQ|SPI|GRBM|CPC|CPF)_[A-Z0-9_]+$", n)]
    idle = scan(P, names, 0.02)
    load = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mfma", "--seconds", "30"],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        time.sleep(6)
        loaded = scan(P, names, 0.02)
    finally:
        load.wait(60)
    print(json.dumps({n: [idle[n], loaded[n]] for n in names}))


if __name__ == "__main__":
    main()
