#!/usr/bin/env python3
"""The reference's collection method, measured on MI355X: one vendor-CLI subprocess per query per
cycle, against gpumon's in-process tick on the same GPU under the same load.

The reference ran `nvidia-smi --query-gpu=...` for device utilisation / memory and
`nvidia-smi --query-compute-apps=...` for the process list every cycle (/root/reference/gpu.py:104-116),
plus 2 docker commands and one `docker top` per container (gpu.py:92-103,177). Its cycle period was
13-19 s in its own screenshots. Neither nvidia-smi nor docker exist here, so this tool
runs the ROCm CLI equivalents of the two GPU queries -- `amd-smi metric` (usage + memory) and
`amd-smi process` -- and times them: a lower bound on the reference design's cycle on this GPU
(docker commands excluded). Then it runs gpumon's exporter in this process for the same number of
ticks and reports its tick.

    python tools/cli_baseline.py --cycles 10 > out.json
"""

import argparse
import json
import os
import resource
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

AMD_SMI = "/opt/rocm/bin/amd-smi"
# the first argv that exits 0 on this image's amd-smi is used (flag spellings vary across releases)
QUERIES = {
    "device_metric": [[AMD_SMI, "metric", "-g", "0", "--usage", "--mem-usage", "--json"],
                      [AMD_SMI, "metric", "-g", "0", "-u", "-m", "--json"],
                      [AMD_SMI, "metric", "-g", "0", "--json"]],
    "process_list": [[AMD_SMI, "process", "-g", "0", "--json"],
                     [AMD_SMI, "process", "--json"]],
}


def _run(argv, timeout=120):
    r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    t0 = time.perf_counter()
    p = subprocess.run(argv, capture_output=True, text=True, timeout=timeout)
    wall = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    return p.returncode, wall, cpu, p.stdout, p.stderr


def _q(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--cycles", type=int, default=10)
    ap.add_argument("--load", default="mixed", choices=["mixed", "idle"])
    a = ap.parse_args()

    load = None
    if a.load != "idle":
        from gpumon.ops.load import SyntheticLoad

        load = SyntheticLoad(0, a.load, hbm_bytes=1 << 30).start()
        time.sleep(2.0)
    out = {"cycles": a.cycles, "load": a.load, "queries": {}}
    try:
        chosen = {}
        for name, cands in QUERIES.items():
            errs = []
            for argv in cands:
                rc, wall, cpu, so, se = _run(argv)
                if rc == 0:
                    chosen[name] = argv
                    out["queries"][name] = {"argv": " ".join(argv[1:]), "first_call_s": round(wall, 3),
                                            "stdout_bytes": len(so)}
                    break
                errs.append(f"{' '.join(argv[1:])}: rc {rc}: {se.strip()[-300:]}")
            if name not in chosen:
                out["queries"][name] = {"error": errs}
        per_cycle, per_query = [], {n: {"wall": [], "cpu": []} for n in chosen}
        for _ in range(a.cycles if chosen else 0):
            t0 = time.perf_counter()
            for name, argv in chosen.items():
                rc, wall, cpu, _, _ = _run(argv)
                per_query[name]["wall"].append(wall)
                per_query[name]["cpu"].append(cpu)
            per_cycle.append(time.perf_counter() - t0)
        for name, d in per_query.items():
            out["queries"][name].update({"wall_p50_s": round(_q(d["wall"], 0.5), 3),
                                         "wall_max_s": round(max(d["wall"]), 3),
                                         "cpu_mean_s": round(sum(d["cpu"]) / len(d["cpu"]), 3)})
        if per_cycle:
            out["cli_cycle_p50_s"] = round(_q(per_cycle, 0.5), 3)
            out["cli_cycle_max_s"] = round(max(per_cycle), 3)
            out["cli_samples_per_s_max"] = round(1.0 / _q(per_cycle, 0.5), 3)

        # gpumon on the same GPU, same load, same process
        from gpumon import core

        ex = core().Exporter({"backend": "amdsmi", "devices": [0], "serve_http": False, "interval_s": 0.1,
                              "log_level": "warn"})
        err = ex.start()
        if err:
            out["gpumon_error"] = err
        else:
            try:
                ex.wait_for_seq(ex.seq + 3, 30)
                q0 = ex.seq
                ex.wait_for_seq(q0 + max(10, a.cycles), 60)
                ticks = [t for t in ex.tick_log() if t["seq"] > q0]
                d = [t["duration_s"] for t in ticks]
                out["gpumon_ticks"] = len(d)
                out["gpumon_tick_p50_ms"] = round(_q(d, 0.5) * 1e3, 3)
                out["gpumon_tick_max_ms"] = round(max(d) * 1e3, 3)
                out["gpumon_rows"] = len([r for r in ex.pod_rows() if not r["idle"]])
                if per_cycle:
                    out["cli_cycle_over_gpumon_tick"] = round(_q(per_cycle, 0.5) / _q(d, 0.5), 1)
            finally:
                ex.stop()
    finally:
        if load:
            load.stop()
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
