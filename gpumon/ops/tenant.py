"""What the exporter costs the workload it watches (tenant overhead).

The reference intrudes on tenants: ``docker exec`` into the workload container every cycle
(/root/reference/gpu.py:221) and ``docker top`` (gpu.py:177). This exporter claims no host-side
stalls; :func:`measure` puts a number on that.

The TENANT is the K2 load running in this process (one ``SyntheticLoad`` per kind, event-timed
FLOP/s or bytes/s). The EXPORTER is ``bin/gpumon-exporter`` started as a separate process per
condition (the deployment shape: a DaemonSet pod next to the workload pods), scraped once per
second like a Prometheus server would. Conditions are interleaved (A B C D A B C D ...) so clock
and thermal drift land on every condition alike; each window's tenant rate is the event-timed
rate over that window, and the slowdown of a condition is its median rate against the median of
the ``none`` windows.
"""

from __future__ import annotations

import os
import statistics
import subprocess
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
EXPORTER = os.path.join(ROOT, "bin", "gpumon-exporter")

# name -> exporter flags (None = no exporter)
CONDITIONS = {
    "none": None,
    "1hz": ["--interval", "1"],
    "10hz": ["--interval", "0.1"],
    "10hz_pmc_probe": ["--interval", "0.1", "--pmc", "--probe"],
}


class _Exporter:
    def __init__(self, flags, port: int, device: int):
        self.port = port
        cmd = [EXPORTER, "--backend", "amdsmi", "--devices", str(device), "--listen", f"127.0.0.1:{port}",
               "--log-level", "warn", "--no-pod-resources", "--no-cri"] + list(flags)
        self.p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        self.scrapes = 0
        self.errors = 0

    def ready(self, timeout_s: float = 20.0) -> bool:
        deadline = time.time() + timeout_s
        while time.time() < deadline:
            if self.p.poll() is not None:
                return False
            try:
                with urllib.request.urlopen(f"http://127.0.0.1:{self.port}/readyz", timeout=1) as r:
                    if r.status == 200:
                        return True
            except OSError:
                pass
            time.sleep(0.1)
        return False

    def scrape(self):
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{self.port}/metrics", timeout=2) as r:
                r.read()
            self.scrapes += 1
        except OSError:
            self.errors += 1

    def stop(self) -> str:
        self.p.terminate()
        try:
            _, err = self.p.communicate(timeout=20)
        except subprocess.TimeoutExpired:
            self.p.kill()
            _, err = self.p.communicate()
        return (err or "")[-400:]


def _rate(kind: str, s0: dict, s1: dict) -> float:
    """Event-timed tenant rate between two LoadGen stats: TFLOP/s (mfma) or TB/s (hbm)."""
    if kind == "hbm":
        dt = s1["hbm_s"] - s0["hbm_s"]
        return (s1["bytes"] - s0["bytes"]) / dt / 1e12 if dt > 0 else float("nan")
    dt = s1["mfma_s"] - s0["mfma_s"]
    return (s1["flops"] - s0["flops"]) / dt / 1e12 if dt > 0 else float("nan")


def measure(kinds=("mfma", "hbm"), conditions=tuple(CONDITIONS), reps: int = 3, window_s: float = 5.0,
            settle_s: float = 2.0, device: int = 0, port: int = 9471, log=None) -> dict:
    """Interleaved A/B/C/D windows per tenant kind; returns per kind and condition the window
    rates, their median and the slowdown in percent against ``none``."""
    from .load import SyntheticLoad

    out = {"window_s": window_s, "reps": reps, "kinds": {}}
    for kind in kinds:
        res = {c: [] for c in conditions}
        extra = {c: {"scrapes": 0, "scrape_errors": 0} for c in conditions}
        with SyntheticLoad(device, kind) as load:
            time.sleep(settle_s * 2)  # clocks / power settle under the load first
            for r in range(reps):
                for c in conditions:
                    ex = None
                    if CONDITIONS[c] is not None:
                        ex = _Exporter(CONDITIONS[c], port, device)
                        if not ex.ready():
                            raise RuntimeError(f"exporter for {c} did not come up: {ex.stop()}")
                    time.sleep(settle_s)
                    s0 = load.stats()
                    t_end = time.perf_counter() + window_s
                    while time.perf_counter() < t_end:
                        if ex is not None:
                            ex.scrape()
                        time.sleep(min(1.0, max(0.0, t_end - time.perf_counter())))
                    s1 = load.stats()
                    res[c].append(_rate(kind, s0, s1))
                    if ex is not None:
                        extra[c]["scrapes"] += ex.scrapes
                        extra[c]["scrape_errors"] += ex.errors
                        ex.stop()
                    if log:
                        log(f"{kind} rep{r} {c}: {res[c][-1]:.4f}")
        base = statistics.median(res["none"]) if res.get("none") else None
        kd = {}
        for c in conditions:
            med = statistics.median(res[c])
            kd[c] = {"rates": res[c], "median": med,
                     "slowdown_pct": (100.0 * (base - med) / base) if base and c != "none" else 0.0, **extra[c]}
        kd["unit"] = "TB/s" if kind == "hbm" else "TFLOP/s"
        # run-to-run spread of the baseline itself: the noise floor the slowdowns sit in
        if base and len(res["none"]) > 1:
            kd["none_spread_pct"] = 100.0 * (max(res["none"]) - min(res["none"])) / base
        out["kinds"][kind] = kd
    return out
