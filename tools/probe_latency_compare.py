#!/usr/bin/env python3
"""K1 probe latency as exported by bin/gpumon-exporter with the probe in the on-device helper
(ondevice_isolate, the default) and in the exporter process, idle and next to a load process.

    python tools/probe_latency_compare.py [--seconds 6] > out.json
"""

from __future__ import annotations

import argparse
import json
import os
import re
import socket
import statistics
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _series(text, name):
    return [float(m.group(1)) for m in re.finditer(rf"^{name}{{[^}}]*}} (\S+)$", text, re.M)]


def run(isolate, seconds):
    port = _port()
    env = dict(os.environ, GPUMON_ONDEVICE_ISOLATE="true" if isolate else "false")
    ex = subprocess.Popen([os.path.join(ROOT, "bin", "gpumon-exporter"), "--backend", "amdsmi", "--interval", "0.1",
                           "--probe", "--listen", f"127.0.0.1:{port}", "--no-pod-resources", "--no-cri",
                           "--log-level", "warn"], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env, text=True)
    lat, span = [], []
    try:
        time.sleep(3)
        if ex.poll() is not None:
            raise SystemExit(ex.stderr.read()[-2000:])
        end = time.time() + seconds
        while time.time() < end:
            m = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
            lat += _series(m, "gpu_probe_latency_seconds")
            span += _series(m, "gpu_probe_kernel_span_seconds")
            time.sleep(0.1)
    finally:
        ex.terminate()
        ex.wait(20)

    def st(xs):
        xs = [x * 1e6 for x in xs]
        return {"n": len(xs), "median_us": round(statistics.median(xs), 1), "min_us": round(min(xs), 1),
                "max_us": round(max(xs), 1)} if xs else None

    return {"latency": st(lat), "gpu_span": st(span)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6)
    a = ap.parse_args()
    out = {}
    for load in ("idle", "mixed"):
        lp = None
        if load != "idle":
            lp = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", load, "--seconds",
                                   str(4 * a.seconds + 30)], cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            time.sleep(5)
        try:
            for iso in (True, False):
                key = f"{load}/{'helper' if iso else 'in_process'}"
                out[key] = run(iso, a.seconds)
                print(key, out[key], file=sys.stderr, flush=True)
        finally:
            if lp is not None:
                lp.terminate()
                lp.wait(60)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
