#!/usr/bin/env python3
"""Where the tick's process-list phase goes on this box: the same reads SysfsGpu::processes makes
(KFD listing, vram_<gpu_id>, the DRM fds' fdinfo), timed one by one against a child that holds a
HIP context through `gpumon load`. Prints one JSON line (microseconds, medians of --reads passes).
"""

import argparse
import glob
import json
import os
import statistics
import subprocess
import sys
import time

KFD = "/sys/class/kfd/kfd/proc"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def t_us(fn, n):
    xs = []
    for _ in range(n):
        t0 = time.perf_counter_ns()
        fn()
        xs.append((time.perf_counter_ns() - t0) / 1e3)
    return round(statistics.median(xs), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=500)
    a = ap.parse_args()
    child = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mfma", "--seconds", "20"], cwd=ROOT,
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        time.sleep(8)
        gid = None
        for p in glob.glob(f"{KFD}/{child.pid}/vram_*"):
            gid = p.rsplit("_", 1)[1]
        fds = []
        for fd in os.listdir(f"/proc/{child.pid}/fd"):
            try:
                if os.readlink(f"/proc/{child.pid}/fd/{fd}").startswith("/dev/dri/"):
                    fds.append(fd)
            except OSError:
                pass
        all_fds = len(os.listdir(f"/proc/{child.pid}/fd"))

        def rd(path):
            with open(path, "rb") as f:
                f.read(4096)

        out = {"child_gpu_id": gid, "kfd_entries": len(os.listdir(KFD)), "child_fds": all_fds,
               "child_drm_fds": len(fds)}
        out["kfd_listdir_us"] = t_us(lambda: os.listdir(KFD), a.reads)
        if gid:
            out["vram_read_us"] = t_us(lambda: rd(f"{KFD}/{child.pid}/vram_{gid}"), a.reads)
            out["cu_occupancy_read_us"] = t_us(lambda: rd(f"{KFD}/{child.pid}/stats_{gid}/cu_occupancy"), a.reads)
        if fds:
            out["fdinfo_read_us_each"] = t_us(lambda: rd(f"/proc/{child.pid}/fdinfo/{fds[0]}"), a.reads)
            out["fdinfo_read_us_all"] = t_us(lambda: [rd(f"/proc/{child.pid}/fdinfo/{x}") for x in fds], a.reads // 5)
        out["stat_read_us"] = t_us(lambda: rd(f"/proc/{child.pid}/stat"), a.reads)
        print(json.dumps(out))
    finally:
        child.terminate()
        child.wait(30)


if __name__ == "__main__":
    main()
