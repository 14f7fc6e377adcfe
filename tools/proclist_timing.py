#!/usr/bin/env python3
"""The tick's process-list phase in isolation on this box: Backend::processes() of GPU 0 timed
back to back (Exporter.time_process_lists) while a `gpumon load` child holds the GPU, with the
real /proc and with procfs pointed at an empty directory (no fdinfo / fd-table reads), so the
split between the KFD sysfs reads and the /proc reads shows. One JSON line."""

import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(procfs):
    from gpumon import core

    cfg = {"backend": "amdsmi", "serve_http": False, "interval_s": 0, "host": "n", "sample_threads": 0,
           "log_level": "warn"}
    if procfs:
        cfg["procfs_root"] = procfs
    ex = core().Exporter(cfg)
    ex.start()
    try:
        r = ex.time_process_lists(0, 300)
    finally:
        ex.stop()
    us = sorted(r["us"][20:])
    return {"rows": r["rows"], "p50_us": round(statistics.median(us), 1), "p10_us": round(us[len(us) // 10], 1),
            "p90_us": round(us[9 * len(us) // 10], 1)}


def main():
    child = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mfma", "--seconds", "25"], cwd=ROOT,
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        time.sleep(8)
        out = {"kfd_entries": len(os.listdir("/sys/class/kfd/kfd/proc"))}
        out["real_proc"] = run(None)
        with tempfile.TemporaryDirectory() as d:
            out["empty_proc"] = run(d)
        out["real_proc_again"] = run(None)
        print(json.dumps(out))
    finally:
        child.terminate()
        child.wait(30)


if __name__ == "__main__":
    main()
