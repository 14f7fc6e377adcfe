#!/usr/bin/env python3
"""Semantics of the gpu_metrics v1.8 per-XCC accumulators (xcp_stats[0]) on MI355X: read the raw
sysfs table twice, 1 s apart, idle and under the bf16 burn, and print delta / delta(accumulation_counter)
for gfx_busy_acc, gfx_below_host_limit_{ppt,thm,total}_acc and gfx_low_utilization_acc."""

import json
import os
import struct
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

FIELDS = {"gfx_busy_acc": 120, "below_ppt": 184, "below_thm": 248, "low_util": 312, "below_total": 376}


def read(path):
    b = open(path, "rb").read()
    acc = struct.unpack_from("<I", b, 40)[0]
    ts = struct.unpack_from("<Q", b, 32)[0]
    x0 = 344
    out = {"acc": acc, "sysclk": ts}
    for k, off in FIELDS.items():
        out[k] = list(struct.unpack_from("<8Q", b, x0 + off))
    out["busy_inst"] = list(struct.unpack_from("<8I", b, x0))
    return out


def delta(a, b):
    dacc = b["acc"] - a["acc"]
    r = {"d_acc": dacc, "dt_s": (b["sysclk"] - a["sysclk"]) / 1e9}
    for k in FIELDS:
        r[k] = [round((y - x) / dacc, 3) if dacc else None for x, y in zip(a[k], b[k])]
    r["busy_inst"] = b["busy_inst"]
    return r


def main():
    from gpumon import core as _core

    core = _core()
    ex = core.Exporter({"backend": "amdsmi", "devices": [0], "serve_http": False, "interval_s": 0})
    ex.start()
    bdf = ex.statics()[0]["bdf"]
    ex.stop()
    path = f"/sys/bus/pci/devices/{bdf}/gpu_metrics"
    out = {"bdf": bdf}
    a = read(path)
    time.sleep(1.0)
    out["idle"] = delta(a, read(path))
    from gpumon.ops.load import SyntheticLoad

    for kind in ("mfma", "hbm"):
        with SyntheticLoad(0, kind):
            time.sleep(1.5)
            a = read(path)
            time.sleep(1.0)
            out[kind] = delta(a, read(path))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
