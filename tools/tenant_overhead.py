#!/usr/bin/env python3
"""Tenant overhead of the exporter on MI355X (gpumon/ops/tenant.py): bf16 MFMA burn TFLOP/s and
HBM stream TB/s, event-timed in the tenant process, with no exporter / 1 Hz / 10 Hz / 10 Hz +
PMC + probe running as a separate process. Prints one JSON document.

    python tools/tenant_overhead.py --reps 3 --window 5 > gpurun_out/x/tenant.json
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gpumon.ops.tenant import CONDITIONS, measure  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="mfma,hbm")
    ap.add_argument("--conditions", default=",".join(CONDITIONS))
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--window", type=float, default=5.0)
    args = ap.parse_args()
    r = measure(kinds=args.kinds.split(","), conditions=args.conditions.split(","), reps=args.reps,
                window_s=args.window, log=lambda m: print(m, file=sys.stderr, flush=True))
    print(json.dumps(r, indent=1))
    for k, kd in r["kinds"].items():
        print(k, {c: (round(v["median"], 3), round(v["slowdown_pct"], 2)) for c, v in kd.items() if isinstance(v, dict)},
              file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
