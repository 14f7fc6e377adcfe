#!/usr/bin/env python3
"""Where the on-device helper's resident memory goes (MI355X): starts bin/gpumon-exporter with the
given flags (default --pmc --probe), then aggregates the helper child's /proc/<pid>/smaps by
mapping (largest first) and reports the totals. Optional --env K=V for the exporter (inherited
by the helper).

    python tools/helper_memory.py [--env GPU_MAX_HW_QUEUES=1] [-- --probe]
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def smaps(pid, top=12):
    agg, cur, tot = {}, None, {"Rss": 0, "Anonymous": 0, "Shared_Clean": 0, "Private_Dirty": 0}
    blocks = []  # individual anonymous mappings >= 8 MB resident (size, rss) in MB
    size = 0
    for line in open(f"/proc/{pid}/smaps"):
        parts = line.split()
        if not parts:
            continue
        if "-" in parts[0] and not parts[0].endswith(":"):
            cur = parts[5] if len(parts) >= 6 else "[anon]"
            lo, hi = (int(x, 16) for x in parts[0].split("-"))
            size = (hi - lo) >> 20
        elif parts[0].rstrip(":") in tot:
            kb = int(parts[1])
            tot[parts[0].rstrip(":")] += kb
            if parts[0] == "Rss:":
                agg[cur] = agg.get(cur, 0) + kb
                if cur == "[anon]" and kb >= 8 << 10:
                    blocks.append((size, round(kb / 1024, 1)))
    return ({k: round(v / 1024, 1) for k, v in tot.items()},
            [(k, round(v / 1024, 1)) for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:top]],
            sorted(blocks, key=lambda b: -b[1]))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("flags", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    flags = [f for f in a.flags if f != "--"] or ["--pmc", "--probe"]
    env = dict(os.environ, **dict(kv.split("=", 1) for kv in a.env))
    ex = subprocess.Popen([os.path.join(ROOT, "bin", "gpumon-exporter"), "--backend", "amdsmi", "--listen",
                           "127.0.0.1:0", "--interval", "1", "--log-level", "warn", "--no-pod-resources", "--no-cri",
                           *flags], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(8)
        if ex.poll() is not None:
            raise SystemExit(ex.stderr.read()[-2000:])
        kids = [int(p) for p in os.listdir("/proc") if p.isdigit() and
                open(f"/proc/{p}/stat").read().rsplit(")", 1)[1].split()[1] == str(ex.pid)]
        out = {"flags": flags, "env": a.env}
        for k in kids:
            tot, top, blocks = smaps(k)
            out[f"helper_{k}"] = {"totals_mb": tot, "top_mappings_mb": top, "anon_blocks_mb": blocks,
                                  "threads": len(os.listdir(f"/proc/{k}/task"))}
        print(json.dumps(out, indent=1))
    finally:
        ex.terminate()
        ex.wait(20)
    return 0


if __name__ == "__main__":
    sys.exit(main())
