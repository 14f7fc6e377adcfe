#!/usr/bin/env python3
"""Time the raw sysfs/KFD reads behind the amdsmi calls the sampler makes, to see where the
per-device sampling cost (gpu_metrics ~0.86 ms, vram ~0.23 ms, process list ~0.54 ms through
libamd_smi on MI355X) actually goes. Prints one JSON object."""

import glob
import json
import os
import statistics
import time


def timed(fn, n=50):
    ts = []
    out = None
    for _ in range(n):
        t = time.perf_counter_ns()
        out = fn()
        ts.append(time.perf_counter_ns() - t)
    return out, {"p50_us": statistics.median(ts) / 1e3, "min_us": min(ts) / 1e3, "max_us": max(ts) / 1e3}


def read_bytes(p):
    with open(p, "rb") as f:
        return f.read()


def main():
    res = {"cards": []}
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        gm = os.path.join(dev, "gpu_metrics")
        if not os.path.exists(gm):
            continue
        card = {"dev": os.path.realpath(dev)}
        try:
            blob, card["gpu_metrics"] = timed(lambda: read_bytes(gm))
            card["gpu_metrics_bytes"] = len(blob)
            card["gpu_metrics_header"] = list(blob[:4])
        except OSError as e:
            card["gpu_metrics_err"] = str(e)
        for f in ("mem_info_vram_used", "mem_info_vram_total", "gpu_busy_percent", "current_link_speed"):
            p = os.path.join(dev, f)
            if os.path.exists(p):
                try:
                    v, card[f] = timed(lambda: read_bytes(p))
                    card[f]["value"] = v.decode().strip()
                except OSError as e:
                    card[f] = str(e)
        res["cards"].append(card)
        if len(res["cards"]) >= 2:
            break
    procs = glob.glob("/sys/class/kfd/kfd/proc/*")
    res["kfd_procs"] = len(procs)

    def scan():
        out = []
        for p in glob.glob("/sys/class/kfd/kfd/proc/*"):
            for f in glob.glob(p + "/vram_*"):
                try:
                    out.append(read_bytes(f))
                except OSError:
                    pass
        return out

    _, res["kfd_scan"] = timed(scan, 20)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
