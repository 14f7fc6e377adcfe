#!/usr/bin/env python3
"""Process-churn soak: GPU tenants start and exit continuously while the exporter samples the GPU
at 10 Hz and a scraper reads /metrics. Each tenant is its own process with its own HIP context,
VRAM and KFD entry (`python -m gpumon load --kind partial`, alive 2-6 s), at most --max-tenants
at once (a gpurun box allows 16 GPU processes per command).

Once a second the tool compares the exporter's process rows with the tenants it knows to be alive:
  - `missed`: a tenant the KFD has shown holding VRAM for more than --grace seconds that has no
    row (the tool reads /sys/class/kfd/kfd/proc/<pid>/vram_* itself);
  - `stale`: a row whose pid exited more than --grace seconds ago;
  - `active_err`: |gpu_active_processes - live tenants|, only while the tenant set has been stable
    for the sharing window (mfma_exclusive_window_s, 5 s), where the two must agree.
Every --window seconds it prints RSS / fds / threads of the process (the exporter lives in it),
ticks, overruns, errors and the scrape p99, so a leak over many arrivals and departures shows as a
trend (the per-pid state: fdinfo tables, occupancy sub-sample lists, cgroup cache, sharing window).
The reference listed containers and their processes from scratch every cycle with `docker top`
(/root/reference/gpu.py:174-178); here the per-pid state is kept across ticks, so churn is the case
that must not leak.

    python tools/churn_soak.py --minutes 4 > out.json     # one JSON line per window, summary last
"""

import argparse
import json
import os
import random
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def proc_stats():
    rss = 0
    with open("/proc/self/status") as f:
        for l in f:
            if l.startswith("VmRSS:"):
                rss = int(l.split()[1]) * 1024
    return {"rss_mb": round(rss / 2 ** 20, 1), "fds": len(os.listdir("/proc/self/fd")),
            "threads": len(os.listdir("/proc/self/task"))}


def kfd_vram(pid):
    """VRAM the KFD reports for `pid` on any GPU (bytes; 0 when it holds none or has no KFD entry):
    the oracle for 'this tenant must have a row'."""
    d = f"/sys/class/kfd/kfd/proc/{pid}"
    tot = 0
    try:
        for f in os.listdir(d):
            if f.startswith("vram_"):
                try:
                    tot += int(open(os.path.join(d, f)).read().strip() or 0)
                except (OSError, ValueError):
                    pass
    except OSError:
        return 0
    return tot


class Churn:
    """Keeps between 0 and max_tenants tenants alive; the target changes every few seconds."""

    def __init__(self, max_tenants, seed):
        self.max = max_tenants
        self.rng = random.Random(seed)
        self.live = {}      # pid -> (Popen, start time)
        self.exited = {}    # pid -> exit time
        self.started = 0
        self.failed = 0
        self.last_change = time.monotonic()
        self.stop = threading.Event()
        self.mu = threading.Lock()

    def _spawn(self):
        life = self.rng.uniform(2.0, 6.0)
        p = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "partial", "--duty", "0.3",
                              "--period", "0.05", "--seconds", f"{life:.2f}"], cwd=ROOT,
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        with self.mu:
            self.live[p.pid] = (p, time.monotonic())
            self.started += 1
            self.last_change = time.monotonic()

    def _reap(self):
        now = time.monotonic()
        with self.mu:
            for pid, (p, _) in list(self.live.items()):
                rc = p.poll()
                if rc is not None:
                    del self.live[pid]
                    self.exited[pid] = now
                    self.failed += rc != 0
                    self.last_change = now
            for pid, t in list(self.exited.items()):
                if now - t > 60:
                    del self.exited[pid]

    def run(self):
        target, next_target = 0, 0.0
        while not self.stop.is_set():
            now = time.monotonic()
            if now >= next_target:
                target = self.rng.randint(0, self.max)
                next_target = now + self.rng.uniform(3.0, 10.0)
            self._reap()
            with self.mu:
                n = len(self.live)
            if n < target:
                self._spawn()
            time.sleep(0.1)

    def drain(self, timeout=30.0):
        self.stop.set()
        end = time.monotonic() + timeout
        while time.monotonic() < end:
            self._reap()
            with self.mu:
                if not self.live:
                    return True
            time.sleep(0.1)
        with self.mu:
            for p, _ in self.live.values():
                p.kill()
        return False


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--minutes", type=float, default=4.0)
    ap.add_argument("--interval", type=float, default=0.1)
    ap.add_argument("--max-tenants", type=int, default=6)
    ap.add_argument("--scrape-rate", type=float, default=20.0)
    ap.add_argument("--window", type=float, default=30.0)
    ap.add_argument("--grace", type=float, default=2.0,
                    help="seconds a tenant may hold VRAM without a row, or a departed pid may keep its row")
    ap.add_argument("--backend", default="amdsmi")
    ap.add_argument("--seed", type=int, default=3)
    a = ap.parse_args()
    if a.max_tenants > 14:
        raise SystemExit("at most 14 tenants (16 GPU processes per gpurun command)")

    from gpumon import core as _core
    from gpumon.config import Config
    from gpumon.export import promtext
    from gpumon.monitor import GpuMonitor

    core = _core()
    cfg = Config(backend=a.backend, devices=[0] if a.backend.startswith("amdsmi") else [], interval=a.interval,
                 listen="127.0.0.1:0", log_level="warn")
    mon = GpuMonitor(cfg, control_plane=False).start()
    if mon.start_error:
        raise SystemExit(mon.start_error)
    churn = Churn(a.max_tenants, a.seed)
    ct = threading.Thread(target=churn.run, daemon=True)
    ct.start()

    scr = {"lat": [], "errors": 0}
    scr_stop = threading.Event()

    def scraper():
        while not scr_stop.is_set():
            r = core.scrape_load("127.0.0.1", mon.port, "/metrics", n_requests=0, duration_s=1.0, concurrency=1,
                                 rate_hz=a.scrape_rate, keep_alive=True, gzip=True)
            scr["lat"].extend(r.get("latencies_s", []))
            scr["errors"] += r.get("errors", 0)

    st_th = threading.Thread(target=scraper, daemon=True)
    st_th.start()

    windows = []
    checks = {"checks": 0, "missed": 0, "stale": 0, "active_checks": 0, "active_err": 0, "rows_max": 0,
              "live_max": 0}
    vram_since = {}  # live tenant pid -> first check that saw it holding VRAM (KFD)
    t_start = time.monotonic()
    end = t_start + a.minutes * 60
    next_win = t_start + a.window
    while time.monotonic() < end:
        time.sleep(1.0)
        now = time.monotonic()
        rows = [r for r in mon.ex.pod_rows() if not r["idle"] and r["dev"] == 0]
        row_pids = {int(r["pid"]) for r in rows if r["pid"].isdigit()}
        with churn.mu:
            live = {pid: t for pid, (_, t) in churn.live.items()}
            exited = dict(churn.exited)
            stable = now - churn.last_change
        checks["checks"] += 1
        checks["rows_max"] = max(checks["rows_max"], len(row_pids))
        checks["live_max"] = max(checks["live_max"], len(live))
        for pid in live:
            if pid not in vram_since and kfd_vram(pid) > 0:
                vram_since[pid] = now
        checks["missed"] += sum(1 for pid, t in vram_since.items()
                                if pid in live and now - t > a.grace and pid not in row_pids)
        for pid in [p for p in vram_since if p not in live]:
            del vram_since[p]
        checks["stale"] += sum(1 for pid in row_pids if pid in exited and now - exited[pid] > a.grace)
        if stable > 5.0 + 2 * a.grace:
            fam = promtext.parse(mon.metrics())
            act = promtext.values(fam, "gpu_active_processes", gpu_id="0")
            checks["active_checks"] += 1
            checks["active_err"] += int(abs((act[0] if act else 0) - len(live)) > 0.5)
        if now >= next_win:
            next_win += a.window
            st = mon.ex.self_stats()
            lat = sorted(scr["lat"])
            scr["lat"] = []
            w = dict(proc_stats(), t_min=round((now - t_start) / 60, 2), ticks=st["ticks"], overruns=st["overruns"],
                     errors=sum(st.get("device_errors", [])), timeouts=sum(st.get("device_timeouts", [])),
                     tenants_started=churn.started, tenants_failed=churn.failed, scrapes=len(lat),
                     scrape_errors=scr["errors"],
                     scrape_p99_ms=round(lat[int(0.99 * (len(lat) - 1))] * 1e3, 3) if lat else None, **checks)
            windows.append(w)
            print(json.dumps(w), flush=True)
    drained = churn.drain()
    time.sleep(2 * a.grace)
    left = [r["pid"] for r in mon.ex.pod_rows() if not r["idle"] and r["dev"] == 0]
    time.sleep(6.0)  # past the sharing window
    fam = promtext.parse(mon.metrics())
    act = promtext.values(fam, "gpu_active_processes", gpu_id="0")
    scr_stop.set()
    st_th.join(5)
    st = mon.ex.self_stats()
    mon.stop()
    first, last = windows[0] if windows else {}, windows[-1] if windows else {}
    summary = {"minutes": a.minutes, "interval_s": a.interval, "max_tenants": a.max_tenants,
               "tenants_started": churn.started, "tenants_failed": churn.failed, "drained": drained,
               "ticks": st["ticks"], "overruns": st["overruns"], "device_errors": sum(st.get("device_errors", [])),
               **checks, "rows_left_after_drain": left, "active_after_drain": act[0] if act else None,
               "rss_mb_first_window": first.get("rss_mb"), "rss_mb_last_window": last.get("rss_mb"),
               "fds_first_window": first.get("fds"), "fds_last_window": last.get("fds"),
               "threads_last_window": last.get("threads"), "scrape_errors": scr["errors"],
               "scrape_p99_ms_max_window": max((w["scrape_p99_ms"] or 0) for w in windows) if windows else None}
    print(json.dumps(summary), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
