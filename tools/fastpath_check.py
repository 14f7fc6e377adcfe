#!/usr/bin/env python3
"""Validate the amdsmi sysfs/KFD fast path on real hardware and measure what it saves.

1. libamd_smi vs sysfs-decoded gpu_metrics v1.8, field by field (counters may advance between
   the two reads; everything else must match).
2. Process rows: libamd_smi process list vs KFD/fdinfo scan for this process (which holds VRAM).
3. Per-call latency and tick time with the fast path on vs off.
Prints one JSON object.
"""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

COUNTERS = ("energy_accumulator", "system_clock_counter", "firmware_timestamp", "accumulation_counter",
            "_residency_acc", "activity_acc", "gfx_busy_acc", "xgmi_read_data_acc", "xgmi_write_data_acc",
            "pcie_bandwidth_acc", "low_utilization_acc")
NOISY = ("temperature", "power", "clk", "activity", "gfx_busy_inst", "pcie_bandwidth_inst")


def main():
    import torch

    from gpumon import core as _core

    core = _core()
    x = torch.ones(1 << 28, device="cuda")  # 1 GiB so this process shows up with VRAM
    torch.cuda.synchronize()
    out = {}
    r = core.amdsmi_compare_tables("", "/sys", 0)
    out["compare_error"] = r["error"]
    out["fast_path_devices"] = r.get("fast_path_devices")
    out["fast_path_status"] = r.get("fast_path_status")
    mism, counters, noisy = [], [], []
    for name, a, s in r.get("rows", []):
        same = (a != a and s != s) or a == s
        if same:
            continue
        if any(c in name for c in COUNTERS):
            counters.append((name, a, s))
        elif any(c in name for c in NOISY):
            noisy.append((name, a, s))
        else:
            mism.append((name, a, s))
    out["rows"] = len(r.get("rows", []))
    out["mismatches"] = mism
    out["counter_diffs"] = counters[:20]
    out["noisy_diffs"] = noisy[:40]

    res = {}
    for fp in (False, True):
        ex = core.Exporter({"backend": "amdsmi", "devices": [0], "serve_http": False, "interval_s": 0,
                            "fast_path": fp, "verify_kfd": False})
        ex.start()
        ticks = []
        for _ in range(30):
            t = time.perf_counter()
            ex.tick()
            ticks.append((time.perf_counter() - t) * 1e3)
            time.sleep(0.02)
        st = ex.self_stats()
        rows = [r for r in ex.pod_rows() if not r["idle"]]
        sm = ex.samples()[0]
        res["fast" if fp else "amdsmi"] = {
            "fast_path_devices": st["fast_path_devices"],
            "fast_path_status": st["fast_path_status"],
            "tick_ms_p50": sorted(ticks)[len(ticks) // 2],
            "tick_ms_min": min(ticks),
            "call_us": {k: v["seconds"] / max(1, v["n"]) * 1e6 for k, v in st["backend_calls"].items()},
            "procs": sorted((r["pid"], r["used_memory_bytes"], r["cu_occupancy"], r["proc_gfx_util"]) for r in rows),
            "vram_used": sm["fields"]["vram_used"],
            "gtt_used": sm["fields"]["gtt_used"],
            "gfx_util": sm["fields"]["gfx_util"],
            "temp_hotspot": sm["fields"]["temp_hotspot"],
            "n_xcd": len(sm["xcd_busy"]),
        }
        ex.stop()
    out["exporter"] = res
    out["self_pid"] = os.getpid()
    del x
    print(json.dumps(out, indent=1, default=str))


if __name__ == "__main__":
    main()
