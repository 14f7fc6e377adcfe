#!/usr/bin/env python3
"""Exporter footprint in the deployed shape (MI355X): RSS and CPU of each exporter configuration
as its own process, observing an external load process, scraped every 15 s like a Prometheus
server. The numbers set the DaemonSet requests / limits (deploy/k8s/gpumon-daemonset.yaml).

Configurations run side by side (they only read the device; at most one uses the PMC counters):

  native_1hz             bin/gpumon-exporter --interval 1
  native_10hz            bin/gpumon-exporter --interval 0.1
  native_10hz_pmc_probe  bin/gpumon-exporter --interval 0.1 --pmc --probe
  python_1hz             python -m gpumon serve --interval 1      (native control plane, no grpcio)

    python tools/footprint.py --seconds 600 > out.json     (progress lines on stderr every 30 s)
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "bin", "gpumon-exporter")
HZ = os.sysconf("SC_CLK_TCK")
BACKEND = "amdsmi"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _children(pid):
    out = []
    for p in os.listdir("/proc"):
        if p.isdigit():
            try:
                if int(open(f"/proc/{p}/stat").read().rsplit(")", 1)[1].split()[1]) == pid:
                    out.append(int(p))
            except (OSError, ValueError, IndexError):
                pass
    return out


def _proc_tree(pid):
    """_proc summed over pid and its child processes (the PMC helper): the container's footprint."""
    rss, hwm, cpu = _proc(pid)
    for c in _children(pid):
        try:
            r, h, u = _proc(c)
        except OSError:
            continue
        rss, hwm, cpu = rss + r, hwm + h, cpu + u
    return rss, hwm, cpu


def _proc(pid):
    """(rss bytes, peak rss bytes, cpu seconds) of pid and its threads."""
    rss = hwm = 0
    with open(f"/proc/{pid}/status") as fh:
        for line in fh:
            if line.startswith("VmRSS:"):
                rss = int(line.split()[1]) * 1024
            elif line.startswith("VmHWM:"):
                hwm = int(line.split()[1]) * 1024
    with open(f"/proc/{pid}/stat") as fh:
        f = fh.read().rsplit(")", 1)[1].split()
    return rss, hwm, (int(f[11]) + int(f[12])) / HZ


CONFIGS = {
    "native_1hz": lambda port: [EXE, "--backend", BACKEND, "--interval", "1"],
    "native_10hz": lambda port: [EXE, "--backend", BACKEND, "--interval", "0.1"],
    "native_10hz_pmc_probe": lambda port: [EXE, "--backend", BACKEND, "--interval", "0.1", "--pmc", "--probe"],
    "python_1hz": lambda port: [sys.executable, "-m", "gpumon", "serve", "--backend", BACKEND, "--interval", "1"],
}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=600)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--scrape-every", type=float, default=15.0)
    ap.add_argument("--backend", default="amdsmi", help="mock:gpus=8 for a CPU rehearsal (no load process)")
    args = ap.parse_args()
    global BACKEND
    BACKEND = args.backend
    load = None if not BACKEND.startswith("amdsmi") else subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mixed", "--seconds",
                             str(args.seconds + 60)], cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    time.sleep(5)
    procs = {}
    for name in args.configs.split(","):
        port = _port()
        cmd = CONFIGS[name](port) + ["--listen", f"127.0.0.1:{port}", "--log-level", "warn"]
        if name.startswith("native"):
            cmd += ["--no-pod-resources", "--no-cri"]
        procs[name] = {"p": subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                             text=True), "port": port, "cmd": " ".join(cmd[1:] if cmd[0] == EXE else cmd[2:]),
                       "rss": [], "scrapes": 0, "scrape_errors": 0, "scrape_ms": []}
    time.sleep(10)  # start-up (HSA / rocprofiler init) is not steady state
    for name, d in procs.items():
        if d["p"].poll() is not None:
            raise SystemExit(f"{name} exited: {d['p'].stderr.read()[-1500:]}")
        d["cpu0"] = _proc_tree(d["p"].pid)[2]
    t0 = time.time()
    last_scrape = 0.0
    last_log = t0
    while time.time() - t0 < args.seconds:
        now = time.time()
        for name, d in procs.items():
            rss, hwm, cpu = _proc_tree(d["p"].pid)
            d["rss"].append(rss)
            d["hwm"] = hwm
            d["cpu1"] = cpu
        if now - last_scrape >= args.scrape_every:
            last_scrape = now
            for name, d in procs.items():
                t = time.perf_counter()
                try:
                    with urllib.request.urlopen(f"http://127.0.0.1:{d['port']}/metrics", timeout=5) as r:
                        r.read()
                    d["scrapes"] += 1
                    d["scrape_ms"].append((time.perf_counter() - t) * 1e3)
                except OSError:
                    d["scrape_errors"] += 1
        if now - last_log >= 30:
            last_log = now
            el = now - t0
            print(json.dumps({"t": round(el), **{n: {"rss_mb": round(d["rss"][-1] / 2**20, 1),
                                                      "cpu_pct": round(100 * (d["cpu1"] - d["cpu0"]) / el, 2)}
                                                  for n, d in procs.items()}}), file=sys.stderr, flush=True)
        time.sleep(2.0)
    wall = time.time() - t0
    out = {"seconds": round(wall, 1), "backend": BACKEND,
           "load": "gpumon load --kind mixed (separate process)" if load is not None else None, "configs": {}}
    for name, d in procs.items():
        d["p"].terminate()
        try:
            d["p"].wait(20)
        except subprocess.TimeoutExpired:
            d["p"].kill()
        rss = sorted(d["rss"])
        out["configs"][name] = {
            "cmd": d["cmd"],
            "cpu_pct_of_core": round(100 * (d["cpu1"] - d["cpu0"]) / wall, 3),
            "cpu_millicores": round(1000 * (d["cpu1"] - d["cpu0"]) / wall, 1),
            "rss_mb_median": round(rss[len(rss) // 2] / 2**20, 1),
            "rss_mb_max": round(rss[-1] / 2**20, 1),
            "rss_mb_first": round(d["rss"][0] / 2**20, 1),
            "rss_mb_last": round(d["rss"][-1] / 2**20, 1),
            "vm_hwm_mb": round(d.get("hwm", 0) / 2**20, 1),
            "scrapes": d["scrapes"], "scrape_errors": d["scrape_errors"],
            "scrape_ms_max": round(max(d["scrape_ms"]), 3) if d["scrape_ms"] else None,
        }
    if load is not None:
        load.terminate()
        load.wait(60)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
