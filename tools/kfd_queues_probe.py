#!/usr/bin/env python3
"""Which KFD processes hold hardware queues on a GPU (VERDICT r5 What's weak #5 / Next #3).

A multi-GPU process (an RCCL rank, a P2P peer) has a KFD context -- a /sys/class/kfd/kfd/proc/<pid>
entry with vram_<gpu_id> -- on GPUs it never launches work on. The exporter hid such "peer
contexts" by a VRAM threshold. KFD also lists each process's user-mode queues under
``proc/<pid>/queues/<qid>/{gpuid,type,size}``: this tool starts tenants that differ only in what
they did on the GPU and prints what KFD shows for each:

  alloc_only   torch.empty on the device (a context + VRAM, no work)
  copy_only    a pinned host -> device copy, then idle
  kernel_once  one kernel, then idle with its VRAM
  kernels      kernels in a loop

    python tools/kfd_queues_probe.py > out.json
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
import time

KFD = "/sys/class/kfd/kfd/proc"

CHILD = r"""
import sys, time, torch
kind = sys.argv[1]
d = torch.device("cuda:0")
x = torch.empty(int(sys.argv[3]) << 30, dtype=torch.uint8, device=d)  # a distinct size per tenant: KFD lists host pids
if kind == "copy_only":
    h = torch.ones(16 << 20, dtype=torch.uint8, pin_memory=True)
    x[: h.numel()].copy_(h, non_blocking=True)
    torch.cuda.synchronize()
elif kind == "kernel_once":
    x.fill_(1)
    torch.cuda.synchronize()
print("ready", flush=True)
t_end = time.time() + float(sys.argv[2])
a = torch.randn(2048, 2048, device=d) if kind == "kernels" else None
while time.time() < t_end:
    if a is not None:
        a = a @ a
        a = a / a.norm()
        torch.cuda.synchronize()
    else:
        time.sleep(0.05)
"""


def _read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError as e:
        return f"<{e.__class__.__name__}>"


def describe(pid: int):
    base = f"{KFD}/{pid}"
    if not os.path.isdir(base):
        return {"kfd": False}
    ents = sorted(os.listdir(base))
    out = {"kfd": True, "entries": ents, "vram": {e[5:]: _read(f"{base}/{e}") for e in ents if e.startswith("vram_")}}
    qs = []
    qdir = f"{base}/queues"
    t0 = time.perf_counter()
    if os.path.isdir(qdir):
        for q in sorted(os.listdir(qdir)):
            qs.append({"qid": q, **{f: _read(f"{qdir}/{q}/{f}") for f in sorted(os.listdir(f"{qdir}/{q}"))}})
    out["scan_us"] = round((time.perf_counter() - t0) * 1e6, 1)
    out["queues"] = qs
    return out


def main() -> int:
    kinds = ["alloc_only", "copy_only", "kernel_once", "kernels"]
    gib = {k: i + 1 for i, k in enumerate(kinds)}  # 1..4 GiB: the tenant behind a host-pid KFD entry
    procs = {}
    for k in kinds:
        procs[k] = subprocess.Popen([sys.executable, "-c", CHILD, k, "40", str(gib[k])], stdout=subprocess.PIPE,
                                    text=True)
    out = {"gpu_ids": {}, "tenants": {}}
    try:
        for k, p in procs.items():
            line = p.stdout.readline().strip()
            if line != "ready":
                raise SystemExit(f"{k}: child said {line!r}")
        time.sleep(2.0)
        for n in sorted(os.listdir("/sys/class/kfd/kfd/topology/nodes")):
            gid = _read(f"/sys/class/kfd/kfd/topology/nodes/{n}/gpu_id")
            if gid not in ("0", "") and not gid.startswith("<"):
                out["gpu_ids"][n] = gid
        for k, p in procs.items():
            out["tenants"][k] = {"pid": p.pid, "gib": gib[k], **describe(p.pid)}
        # /sys/class/kfd/kfd/proc lists HOST pids: in a container with its own pid namespace the
        # tenants' entries are found by their VRAM instead (each allocated a distinct size)
        gids = set(out["gpu_ids"].values())
        entries = []
        for e in sorted(os.listdir(KFD)):
            if not e.isdigit():
                continue
            d = describe(int(e))
            vram = [int(v) for g, v in d.get("vram", {}).items() if g in gids and v.isdigit()]
            if not vram:
                continue
            d["kfd_pid"] = int(e)
            d["vram_bytes"] = max(vram)
            near = min(kinds, key=lambda k: abs(d["vram_bytes"] - (gib[k] << 30)))
            d["tenant"] = near if abs(d["vram_bytes"] - (gib[near] << 30)) < (256 << 20) else None
            entries.append(d)
        out["kfd_entries_on_gpu"] = entries
    finally:
        for p in procs.values():
            p.terminate()
        for p in procs.values():
            p.wait(timeout=30)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
