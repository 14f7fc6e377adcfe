#!/usr/bin/env python3
"""What the firmware's PCIe bandwidth fields mean on MI355X (VERDICT r5 What's weak #2).

gpu_metrics v1.8 carries ``pcie_bandwidth_inst`` and ``pcie_bandwidth_acc`` (offsets 96 / 88) next to
``accumulation_counter`` (offset 40) and ``firmware_timestamp`` (offset 288, 10 ns units). The
exporter published the instantaneous one as GB/s and it read 18-35 on idle GPUs. This tool drives
known host<->device traffic (pinned ``copy_`` on their own streams, bytes over wall time) in phases
and reads the raw table every --period ms, so each phase gives the firmware's numbers next to the
traffic's real rate:

    idle / h2d / d2h / bidir / h2d_half (50 % duty) / idle

    python tools/pcie_probe.py [--phase-s 3] [--mb 512] > out.json

Per phase: copy GB/s (host clock), mean ``inst``, d(acc)/d(accumulation_counter),
d(acc)/d(firmware seconds) and the table count; ratios against the copy rate say which unit holds.
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import struct
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _metrics_path(bdf: str | None):
    if bdf:
        return f"/sys/bus/pci/devices/{bdf}/gpu_metrics"
    for p in sorted(glob.glob("/sys/class/drm/card*/device/gpu_metrics")):
        try:
            with open(p, "rb") as fh:
                if len(fh.read()) > 4:
                    return os.path.realpath(p)
        except OSError:
            continue
    raise SystemExit("no readable gpu_metrics file")


def _read(fd):
    b = os.pread(fd, 65536, 0)
    if (b[2], b[3]) != (1, 8):
        raise SystemExit(f"gpu_metrics v{b[2]}.{b[3]}: offsets known for v1.8 only")
    return {"acc_counter": struct.unpack_from("<I", b, 40)[0],
            "pcie_acc": struct.unpack_from("<Q", b, 88)[0],
            "pcie_inst": struct.unpack_from("<Q", b, 96)[0],
            "fw_ts": struct.unpack_from("<Q", b, 288)[0],
            "sys_ns": struct.unpack_from("<Q", b, 32)[0],
            "width": struct.unpack_from("<H", b, 68)[0],
            "speed": struct.unpack_from("<H", b, 70)[0],
            "t": time.perf_counter()}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--phase-s", type=float, default=3.0)
    ap.add_argument("--mb", type=int, default=512)
    ap.add_argument("--period", type=float, default=20.0, help="ms between table reads")
    ap.add_argument("--bdf", default=None)
    args = ap.parse_args()

    import torch

    dev = torch.device("cuda:0")
    bdf = args.bdf
    if bdf is None:
        from gpumon.parallel.devmap import hip_bdfs

        bdf = hip_bdfs([0]).get(0)
    path = _metrics_path(bdf)
    fd = os.open(path, os.O_RDONLY)
    n = args.mb << 20
    h_src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(n, dtype=torch.uint8, device=dev)
    d_b = torch.empty(n, dtype=torch.uint8, device=dev)
    s_up, s_down = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()

    moved = {"h2d": 0, "d2h": 0}
    stop = threading.Event()

    def run(kind, duty):
        while not stop.is_set():
            t0 = time.perf_counter()
            if kind in ("h2d", "bidir"):
                with torch.cuda.stream(s_up):
                    d_a.copy_(h_src, non_blocking=True)
            if kind in ("d2h", "bidir"):
                with torch.cuda.stream(s_down):
                    h_dst.copy_(d_b, non_blocking=True)
            s_up.synchronize()
            s_down.synchronize()
            if kind in ("h2d", "bidir"):
                moved["h2d"] += n
            if kind in ("d2h", "bidir"):
                moved["d2h"] += n
            if duty < 1.0:
                time.sleep((time.perf_counter() - t0) * (1.0 / duty - 1.0))

    out = {"path": path, "bdf": bdf, "mb": args.mb, "phases": []}
    for f in ("current_link_speed", "current_link_width", "max_link_speed", "max_link_width"):
        try:
            out[f] = open(os.path.join(os.path.dirname(path), f)).read().strip()
        except OSError:
            out[f] = None
    out["pcie_bw_file"] = os.path.exists(os.path.join(os.path.dirname(path), "pcie_bw"))
    for name, kind, duty in (("idle", None, 1.0), ("h2d", "h2d", 1.0), ("d2h", "d2h", 1.0), ("bidir", "bidir", 1.0),
                             ("h2d_half", "h2d", 0.5), ("idle_end", None, 1.0)):
        stop.clear()
        moved["h2d"] = moved["d2h"] = 0
        th = threading.Thread(target=run, args=(kind, duty), daemon=True) if kind else None
        if th:
            th.start()
        time.sleep(0.3)  # settle: the first copies and one firmware period stay out
        m0 = dict(moved)
        t0 = time.perf_counter()
        reads = []
        while time.perf_counter() - t0 < args.phase_s:
            reads.append(_read(fd))
            time.sleep(args.period / 1e3)
        t1 = time.perf_counter()
        m1 = dict(moved)
        stop.set()
        if th:
            th.join()
        torch.cuda.synchronize()
        a, b = reads[0], reads[-1]
        tables = len({r["fw_ts"] for r in reads})
        dfw_s = (b["fw_ts"] - a["fw_ts"]) * 1e-8
        dacc = b["pcie_acc"] - a["pcie_acc"]
        dcnt = b["acc_counter"] - a["acc_counter"]
        gbps = {k: (m1[k] - m0[k]) / (t1 - t0) / 1e9 for k in m1}
        ph = {"phase": name, "seconds": round(t1 - t0, 3), "tables": tables,
              "copy_GBps_h2d": round(gbps["h2d"], 3), "copy_GBps_d2h": round(gbps["d2h"], 3),
              "copy_GBps_total": round(gbps["h2d"] + gbps["d2h"], 3),
              "inst_mean": round(sum(r["pcie_inst"] for r in reads) / len(reads), 3),
              "inst_min": min(r["pcie_inst"] for r in reads), "inst_max": max(r["pcie_inst"] for r in reads),
              "d_acc": dacc, "d_acc_counter": dcnt, "d_fw_s": round(dfw_s, 4),
              "acc_per_counter": round(dacc / dcnt, 4) if dcnt else None,
              "acc_per_fw_s": round(dacc / dfw_s, 3) if dfw_s > 0 else None,
              "counter_per_fw_s": round(dcnt / dfw_s, 3) if dfw_s > 0 else None,
              "link": [a["width"], a["speed"]]}
        out["phases"].append(ph)
        print(json.dumps(ph), file=sys.stderr, flush=True)
    os.close(fd)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
