"""What the exporter costs the workload it watches (tenant overhead).

The reference intrudes on tenants: ``docker exec`` into the workload container every cycle
(/root/reference/gpu.py:221) and ``docker top`` (gpu.py:177). This exporter claims no host-side
stalls; :func:`measure` puts a number on that.

The TENANT is the K2 load running in this process (one ``SyntheticLoad`` per kind, event-timed
FLOP/s or bytes/s), or -- kinds ``gemm`` / ``gemm_shared`` -- PyTorch processes running hipBLASLt
bf16 GEMMs back to back (library kernels, not this repo's burns): ``gemm`` one 8192^3 tenant,
event-timed; ``gemm_shared`` an 8192^3 and a 4096^3 tenant on the same GPU, their summed FLOPs
over wall time (the shared-GPU case). The EXPORTER is ``bin/gpumon-exporter`` started as a separate process per
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
    "10hz_noprewarm": ["--interval", "0.1", "--prewarm-ms", "0"],  # prewarm's own share of the cost
    "10hz_occ1": ["--interval", "0.1", "--occ-samples", "1"],  # KFD cu_occupancy sub-sampling's share
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


GEMM_TENANT = r"""
import sys, time, torch
n = int(sys.argv[1])
a = torch.randn(n, n, device="cuda:0", dtype=torch.bfloat16)
b = torch.randn(n, n, device="cuda:0", dtype=torch.bfloat16)
for _ in range(10):
    a @ b
torch.cuda.synchronize()
print("ready", flush=True)
batch = max(1, int(2 * (8192 / n) ** 3))  # ~1.6 ms of GEMMs per event pair at any size
while True:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(batch):
        a @ b
    e1.record()
    e1.synchronize()
    print(time.time(), 2.0 * n ** 3 * batch, e0.elapsed_time(e1), flush=True)
"""


class GemmTenants:
    """PyTorch hipBLASLt bf16 GEMM tenants in their own processes; stats() mirrors LoadGen.stats()
    for _rate(): cumulative FLOPs and either the event-timed GPU seconds (one tenant) or the wall
    seconds since start (several tenants: their combined throughput over wall time)."""

    def __init__(self, sizes=(8192,), device: int = 0):
        import sys
        import threading

        env = dict(os.environ, HIP_VISIBLE_DEVICES=str(device))
        self.procs = [subprocess.Popen([sys.executable, "-c", GEMM_TENANT, str(n)], stdout=subprocess.PIPE,
                                       stderr=subprocess.PIPE, text=True, env=env) for n in sizes]
        self.flops = 0.0
        self.gpu_s = 0.0
        self.lock = threading.Lock()
        self.ready = 0
        self.t0 = None
        self.threads = [threading.Thread(target=self._read, args=(p,), daemon=True) for p in self.procs]
        for t in self.threads:
            t.start()

    def _read(self, p):
        for line in p.stdout:
            if line.startswith("ready"):
                with self.lock:
                    self.ready += 1
                continue
            _, fl, ms = line.split()
            with self.lock:
                self.flops += float(fl)
                self.gpu_s += float(ms) * 1e-3

    def wait_ready(self, timeout_s: float = 240.0) -> None:
        deadline = time.time() + timeout_s
        while self.ready < len(self.procs):
            if any(p.poll() is not None for p in self.procs) or time.time() > deadline:
                errs = " | ".join((p.stderr.read() or "")[-300:] for p in self.procs if p.poll() is not None)
                raise RuntimeError(f"GEMM tenant did not start: {errs}")
            time.sleep(0.1)
        self.t0 = time.perf_counter()

    def stats(self) -> dict:
        with self.lock:
            wall = time.perf_counter() - (self.t0 or time.perf_counter())
            # one tenant: event-timed (GPU-busy) seconds; several: wall seconds
            return {"flops": self.flops, "mfma_s": self.gpu_s if len(self.procs) == 1 else wall}

    def __enter__(self):
        self.wait_ready()
        return self

    def __exit__(self, *exc):
        for p in self.procs:
            p.kill()
        for p in self.procs:
            p.wait(30)


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
        tenant = (GemmTenants((8192,), device) if kind == "gemm" else
                  GemmTenants((8192, 4096), device) if kind == "gemm_shared" else SyntheticLoad(device, kind))
        with tenant as load:
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
