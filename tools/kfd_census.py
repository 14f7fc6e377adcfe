#!/usr/bin/env python3
"""How many KFD processes does this host list, and what does one pass over them cost?

/sys/class/kfd/kfd/proc is not namespaced: a container sees every KFD process of the host, on
every GPU. The exporter's process list (and its between-tick occupancy scans) try each entry's
vram_<gpu_id> for their own GPU, so a shared host's other tenants cost open() attempts per tick.
Prints one JSON line: entries, entries on this container's GPU(s), and the pass time.
"""

import glob
import json
import os
import time

KFD = "/sys/class/kfd/kfd/proc"


def main():
    ids = set()
    for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            ids.add(int(open(p).read().strip() or 0))
        except (OSError, ValueError):  # GPUs outside this container's device cgroup
            pass
    ids = sorted(ids - {0})  # CPU nodes read 0
    out = {"gpu_ids": ids}
    t0 = time.perf_counter()
    pids = [d for d in os.listdir(KFD) if d.isdigit()] if os.path.isdir(KFD) else []
    t1 = time.perf_counter()
    tries = 0
    for gid in ids[:1]:
        for p in pids:
            tries += 1
            try:
                with open(f"{KFD}/{p}/vram_{gid}") as f:
                    f.read()
            except OSError:
                pass
    t2 = time.perf_counter()
    per_gpu = {}
    for p in pids:
        try:
            for e in os.listdir(f"{KFD}/{p}"):
                if e.startswith("vram_"):
                    per_gpu[e[5:]] = per_gpu.get(e[5:], 0) + 1
        except OSError:
            pass
    out.update(kfd_entries=len(pids), processes_per_gpu_id=per_gpu, listdir_us=round((t1 - t0) * 1e6, 1),
               vram_pass_us=round((t2 - t1) * 1e6, 1), per_try_us=round((t2 - t1) * 1e6 / max(1, tries), 2))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
