#!/usr/bin/env python3
"""K1 probe through lib/libgpumon_probe.so with one launch path per process (GPUMON_PROBE_RUNTIME
= hsa | hip, csrc/plugins/probe_plugin.cpp): N launches, what they measured, and what the process
holds afterwards (resident memory, the ~173 MB per-queue context-save blocks).

    python tools/probe_runtime_check.py [--launches 20] [--runtimes hsa,hip]   # one JSON line each

Each runtime runs in a child process of its own (the choice is made once per process, and a
process that has touched HIP has HIP's queues), so the memory numbers compare like with like.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_XCC = 16


class ProbeResult(ctypes.Structure):  # gpumon_probe_result_t (csrc/plugins/ondevice_abi.h)
    _fields_ = [("seq", ctypes.c_uint32), ("blocks", ctypes.c_int32), ("arrived", ctypes.c_int32),
                ("host_latency_s", ctypes.c_double), ("gpu_span_s", ctypes.c_double),
                ("unique_cus", ctypes.c_int32), ("stale_records", ctypes.c_int32),
                ("xcc_blocks", ctypes.c_int32 * MAX_XCC), ("xcc_clock_mhz", ctypes.c_double * MAX_XCC),
                ("xcc_wave_slot", ctypes.c_double * MAX_XCC), ("wave_slot_mean", ctypes.c_double)]


def _memory():
    """Resident MB of this process and its anonymous mappings of >= 100 MB resident."""
    rss, big, cur_anon, size = 0, [], False, 0
    for line in open("/proc/self/smaps"):
        parts = line.split()
        if parts and "-" in parts[0] and not parts[0].endswith(":"):
            cur_anon = len(parts) < 6
            lo, hi = (int(x, 16) for x in parts[0].split("-"))
            size = (hi - lo) >> 20
        elif parts and parts[0] == "Rss:":
            kb = int(parts[1])
            rss += kb
            if cur_anon and kb >= 100 << 10:
                big.append(round(kb / 1024, 1))
    return round(rss / 1024, 1), sorted(big, reverse=True)


def child(launches: int, blocks: int) -> dict:
    lib = ctypes.CDLL(os.path.join(ROOT, "lib", "libgpumon_probe.so"))
    lib.gpumon_probe_runtime.restype = ctypes.c_char_p
    lib.gpumon_probe_create.restype = ctypes.c_void_p
    lib.gpumon_probe_create.argtypes = [ctypes.c_int] * 4 + [ctypes.c_char_p, ctypes.c_size_t]
    lib.gpumon_probe_launch.argtypes = [ctypes.c_void_p]
    lib.gpumon_probe_wait.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.POINTER(ProbeResult)]
    lib.gpumon_probe_destroy.argtypes = [ctypes.c_void_p]
    buf = ctypes.create_string_buffer(256)
    lib.gpumon_probe_device_arch.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    lib.gpumon_probe_device_arch(0, buf, 256)
    out = {"runtime": lib.gpumon_probe_runtime().decode(), "devices": lib.gpumon_probe_device_count(),
           "arch": buf.value.decode()}
    rss0, _ = _memory()
    err = ctypes.create_string_buffer(512)
    t0 = time.perf_counter()
    h = lib.gpumon_probe_create(0, blocks, 4, 200, err, 512)  # 2 us spin, 4 slots (the sampler's shape)
    if not h:
        out["error"] = err.value.decode()
        return out
    out["create_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    lat, span, ok, stale, xcc_min, cus = [], [], 0, 0, 1 << 30, 0
    clocks = []
    for _ in range(launches):
        slot = lib.gpumon_probe_launch(h)
        r = ProbeResult()
        if slot < 0 or not lib.gpumon_probe_wait(h, slot, 5.0, ctypes.byref(r)):
            continue
        ok += 1
        lat.append(r.host_latency_s * 1e6)
        span.append(r.gpu_span_s * 1e6)
        stale += r.stale_records
        x = [r.xcc_blocks[k] for k in range(8)]
        xcc_min = min(xcc_min, min(x))
        cus = max(cus, r.unique_cus)
        clocks.append([round(r.xcc_clock_mhz[k]) for k in range(8)])
    rss1, big = _memory()
    lib.gpumon_probe_destroy(h)
    lat.sort()
    out.update({"launches": launches, "complete": ok, "stale_records": stale, "min_blocks_per_xcd": xcc_min,
                "unique_cus": cus, "latency_us_p50": round(lat[len(lat) // 2], 1) if lat else None,
                "latency_us_max": round(lat[-1], 1) if lat else None,
                "kernel_span_us_p50": round(sorted(span)[len(span) // 2], 1) if span else None,
                "xcd_clock_mhz_last": clocks[-1] if clocks else None,
                "rss_mb_before_create": rss0, "rss_mb": rss1, "anon_blocks_ge_100mb": big})
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=1024)
    ap.add_argument("--runtimes", default="hsa,hip")
    ap.add_argument("--child", default="")
    a = ap.parse_args()
    if a.child:
        print(json.dumps(child(a.launches, a.blocks)), flush=True)
        return 0
    rc = 0
    for rt in a.runtimes.split(","):
        env = dict(os.environ, GPUMON_PROBE_RUNTIME=rt)
        r = subprocess.run([sys.executable, __file__, "--child", rt, "--launches", str(a.launches),
                            "--blocks", str(a.blocks)], env=env, capture_output=True, text=True, timeout=120)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else json.dumps(
            {"runtime": rt, "error": f"exit {r.returncode}: {r.stderr[-1500:]}"})
        print(line, flush=True)
        rc = rc or r.returncode
    return rc


if __name__ == "__main__":
    sys.exit(main())
