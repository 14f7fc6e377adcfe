#!/usr/bin/env python3
"""How KFD ``stats_<gpu_id>/cu_occupancy`` behaves under the K2 loads (MI355X hardware probe).

For each load kind, starts ``python -m gpumon load --kind K`` as a CHILD process (the deployment
shape: exporter and tenant are different processes), then reads the child's
``/sys/class/kfd/kfd/proc/<pid>/stats_<gpu_id>/cu_occupancy`` as fast as it can for ``--seconds``
and prints the distribution (and the read cost), plus the other files KFD exposes for the pid.

    python tools/kfd_occupancy_probe.py --kinds mfma,hbm,mixed,concurrent,partial,self-mfma --seconds 2 > out.json
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KFD = "/sys/class/kfd/kfd/proc"


def _read(path):
    try:
        with open(path, "rb") as fh:
            return fh.read().decode(errors="replace").strip()
    except OSError as e:
        return f"ERR {e.errno}"


def _kfd_pids():
    try:
        return set(os.listdir(KFD))
    except OSError:
        return set()


def find_kfd_entry(before: set, timeout_s: float = 30.0):
    """KFD names its proc entries by HOST pid; inside a container's pid namespace the child's pid
    differs, so the child's entry is the one that appears after it starts and holds VRAM."""
    deadline = time.time() + timeout_s
    while time.time() < deadline:
        for e in sorted(_kfd_pids() - before):
            for v in glob.glob(f"{KFD}/{e}/vram_*"):
                try:
                    if int(_read(v)) > (256 << 20):
                        return int(e)
                except ValueError:
                    pass
        time.sleep(0.1)
    return None


def probe_pid(pid: int, seconds: float) -> dict:
    pdir = f"{KFD}/{pid}"
    files = sorted(os.path.relpath(p, pdir) for p in glob.glob(pdir + "/**", recursive=True))
    occ_files = glob.glob(pdir + "/stats_*/cu_occupancy")
    out = {"pid": pid, "files": files, "static": {f: _read(os.path.join(pdir, f)) for f in files
                                                    if os.path.isfile(os.path.join(pdir, f))
                                                    and "cu_occupancy" not in f}}
    if not occ_files:
        out["error"] = "no cu_occupancy file"
        return out
    f = occ_files[0]
    time.sleep(1.0)  # let the load reach steady state
    vals, costs = [], []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        t0 = time.perf_counter()
        v = _read(f)
        costs.append(time.perf_counter() - t0)
        try:
            vals.append(int(v))
        except ValueError:
            vals.append(-1)
    nz = [v for v in vals if v > 0]
    out.update({"file": os.path.relpath(f, pdir), "reads": len(vals),
                "mean": statistics.fmean(vals) if vals else None,
                "nonzero_frac": len(nz) / max(1, len(vals)),
                "min": min(vals) if vals else None, "max": max(vals) if vals else None,
                "hist": {str(k): vals.count(k) for k in sorted(set(vals))[:40]},
                "read_us_p50": statistics.median(costs) * 1e6 if costs else None,
                "read_us_max": max(costs) * 1e6 if costs else None})
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="mfma,hbm,mixed")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--duty", type=float, default=1.0)
    args = ap.parse_args()
    res = []
    print(json.dumps({"kfd_entries": sorted(_kfd_pids()), "self_pid": os.getpid()}), file=sys.stderr)
    for kind in args.kinds.split(","):
        if kind.startswith("self-"):  # the load inside this very process (the bench's shape)
            sys.path.insert(0, ROOT)
            from gpumon.ops.load import SyntheticLoad

            before = _kfd_pids()
            with SyntheticLoad(0, kind[5:]) as load:
                hp = find_kfd_entry(before)
                r = probe_pid(hp, args.seconds) if hp else {"error": "no new KFD entry"}
                r["load_stats"] = json.dumps(load.stats())
            r["kind"] = kind
            res.append(r)
            print(json.dumps({k: r.get(k) for k in ("kind", "pid", "reads", "mean", "nonzero_frac", "min", "max",
                                                    "read_us_p50", "error")}), file=sys.stderr, flush=True)
            continue
        before = _kfd_pids()
        child = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", kind, "--duty", str(args.duty),
                                  "--seconds", str(args.seconds + 6)], cwd=ROOT,
                                 stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
        try:
            hp = find_kfd_entry(before)
            r = probe_pid(hp, args.seconds) if hp else {"error": "no new KFD entry"}
        finally:
            out, _ = child.communicate(timeout=120)
        r["kind"] = kind
        r["load_stats"] = out.strip().splitlines()[-1] if out.strip() else None
        res.append(r)
        print(json.dumps({k: r.get(k) for k in ("kind", "pid", "reads", "mean", "nonzero_frac", "min", "max",
                                                "read_us_p50", "error")}),
              file=sys.stderr, flush=True)
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
