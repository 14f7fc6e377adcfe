#!/usr/bin/env python3
"""Read-latency distribution of every kernel file on the exporter's tick path (MI355X).

A `gpumon load` child runs the chosen K2 load; this process re-reads each file N times and prints
p50 / p99 / max per file, so the tick's tail can be pinned on a file:

  gpu_metrics   /sys/bus/pci/devices/<bdf>/gpu_metrics (held fd, pread at 0: SMU table fetch)
  vram_used     /sys/bus/pci/devices/<bdf>/mem_info_vram_used
  kfd_vram      /sys/class/kfd/kfd/proc/<child>/vram_<gpu_id>
  cu_occupancy  /sys/class/kfd/kfd/proc/<child>/stats_<gpu_id>/cu_occupancy
  fdinfo        /proc/<child>/fdinfo/<its render-node fd>
  kfd_listdir   os.listdir(/sys/class/kfd/kfd/proc)

    python tools/sysfs_read_latency.py --kind mixed --reads 2000 > out.json   (--kind idle: a child that
                                                                          only holds a GPU context)
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KFD = "/sys/class/kfd/kfd/proc"


def _bdf_and_gpu_id():
    for node in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*")):
        try:
            gid = int(open(node + "/gpu_id").read())
        except (OSError, ValueError):
            continue
        if not gid:
            continue
        props = dict(l.split()[:2] for l in open(node + "/properties") if len(l.split()) >= 2)
        loc = int(props.get("location_id", "0"))
        dom = int(props.get("domain", "0"))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"
        return bdf, gid
    raise SystemExit("no GPU node in the KFD topology")


def _stats(ns):
    ns = sorted(ns)
    q = lambda p: ns[min(len(ns) - 1, int(p * (len(ns) - 1)))] / 1e3  # noqa: E731
    return {"n": len(ns), "p50_us": round(q(0.5), 1), "p99_us": round(q(0.99), 1), "max_us": round(ns[-1] / 1e3, 1)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="mixed")
    ap.add_argument("--reads", type=int, default=2000)
    a = ap.parse_args()
    bdf, gid = _bdf_and_gpu_id()
    before = set(os.listdir(KFD)) if os.path.isdir(KFD) else set()
    cmd = ([sys.executable, "-c", "import sys, time; sys.path.insert(0, %r); from gpumon import hip; "
            "h = hip(); h.device_count(); time.sleep(120)" % ROOT] if a.kind == "idle" else
           [sys.executable, "-m", "gpumon", "load", "--kind", a.kind, "--seconds", "120"])
    child = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        kpid = None
        for _ in range(300):  # the child's KFD entry (host pid: diff the directory)
            time.sleep(0.1)
            new = [p for p in set(os.listdir(KFD)) - before if os.path.exists(f"{KFD}/{p}/vram_{gid}")]
            if new:
                kpid = new[0]
                break
        if kpid is None:
            raise SystemExit("child never opened the GPU")
        time.sleep(4)  # load running
        dev = f"/sys/bus/pci/devices/{bdf}"
        files = {"gpu_metrics": f"{dev}/gpu_metrics", "vram_used": f"{dev}/mem_info_vram_used",
                 "kfd_vram": f"{KFD}/{kpid}/vram_{gid}", "cu_occupancy": f"{KFD}/{kpid}/stats_{gid}/cu_occupancy"}
        # the child's render-node fd (our pid namespace sees it under child.pid)
        for fd in os.listdir(f"/proc/{child.pid}/fd"):
            try:
                if os.readlink(f"/proc/{child.pid}/fd/{fd}").startswith("/dev/dri/renderD"):
                    files["fdinfo"] = f"/proc/{child.pid}/fdinfo/{fd}"
                    break
            except OSError:
                pass
        out = {"kind": a.kind, "bdf": bdf, "gpu_id": gid, "files": {}}
        held = ("gpu_metrics", "vram_used")  # the exporter holds these open; the rest it opens per read
        for name, path in files.items():
            ns = []
            if name in held:
                fd = os.open(path, os.O_RDONLY)
                try:
                    for _ in range(a.reads):
                        t = time.perf_counter_ns()
                        os.pread(fd, 8192, 0)
                        ns.append(time.perf_counter_ns() - t)
                finally:
                    os.close(fd)
            else:
                for _ in range(a.reads):
                    t = time.perf_counter_ns()
                    fd = os.open(path, os.O_RDONLY)
                    os.read(fd, 8192)
                    os.close(fd)
                    ns.append(time.perf_counter_ns() - t)
            out["files"][name] = _stats(ns)
            print(name, out["files"][name], file=sys.stderr, flush=True)
        ns = []
        for _ in range(a.reads):
            t = time.perf_counter_ns()
            os.listdir(KFD)
            ns.append(time.perf_counter_ns() - t)
        out["files"]["kfd_listdir"] = _stats(ns)
        print(json.dumps(out, indent=1))
    finally:
        child.terminate()
        child.wait(60)
    return 0


if __name__ == "__main__":
    sys.exit(main())
