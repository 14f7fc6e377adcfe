#!/usr/bin/env python3
"""Soak test: the exporter at 10 Hz on the real GPU under the mixed MFMA/HBM load with a
continuous scraper, for --minutes. Every 30 s: RSS, open fds, threads, ticks, overruns, errors,
scrape p99 over the last window. A leak or a slow drift shows up as a trend. One progress line per
window on stdout; the final JSON summary is the last line.
"""

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def proc_stats(pid="self"):
    rss = 0
    with open(f"/proc/{pid}/status") as f:
        for l in f:
            if l.startswith("VmRSS:"):
                rss = int(l.split()[1]) * 1024
    return {"rss_mb": round(rss / 2 ** 20, 1), "fds": len(os.listdir(f"/proc/{pid}/fd")),
            "threads": len(os.listdir(f"/proc/{pid}/task"))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--interval", type=float, default=0.1)
    ap.add_argument("--scrape-rate", type=float, default=50.0)
    ap.add_argument("--backend", default="amdsmi")
    ap.add_argument("--window", type=float, default=30.0)
    ap.add_argument("--child", action="store_true",
                    help="soak the shipped bin/gpumon-exporter as its own process (DaemonSet config keys), "
                         "started before this process's first HIP call; RSS / fds / threads are the child's")
    ap.add_argument("--no-keepalive", action="store_true",
                    help="one connection per scrape (Connection: close): the server's lingering-close path")
    a = ap.parse_args()

    from gpumon import core as _core
    from gpumon.config import Config
    from gpumon.monitor import GpuMonitor

    core = _core()
    real = a.backend.startswith("amdsmi")
    child = None
    if a.child:  # before the load's first HIP call
        import tempfile

        from gpumon.export.child import ChildExporter, daemonset_config
        from gpumon.parallel.devmap import kfd_bdfs

        devs = [kfd_bdfs(range(1))[0]] if real else []
        child = ChildExporter(dict(daemonset_config(), backend=a.backend, devices=devs, interval=a.interval,
                                   log_level="warn", host="soak"), tempfile.mkdtemp(prefix="gpumon-soak-")).start()
    load = None
    if real:
        from gpumon.ops.load import SyntheticLoad

        load = SyntheticLoad(0, "mixed").start()
    if child is None:
        cfg = Config(backend=a.backend, devices=[0] if real else [], interval=a.interval,
                     listen="127.0.0.1:0", log_level="warn")
        mon = GpuMonitor(cfg, control_plane=False).start()
        port, self_stats, pid = mon.port, mon.ex.self_stats, "self"
    else:
        port, self_stats, pid = child.port, child.self_stats, child.pid
    windows = []
    end = time.monotonic() + a.minutes * 60
    base = proc_stats(pid)
    while time.monotonic() < end:
        res = {}

        def scrape():
            res.update(core.scrape_load("127.0.0.1", port, "/metrics", n_requests=0, duration_s=a.window,
                                        concurrency=2, rate_hz=a.scrape_rate, keep_alive=not a.no_keepalive,
                                        gzip=True))

        th = threading.Thread(target=scrape)
        th.start()
        th.join()
        st = self_stats()
        lat = sorted(res.get("latencies_s", []))
        w = dict(proc_stats(pid), t_min=round((a.minutes * 60 - (end - time.monotonic())) / 60, 2),
                 ticks=st["ticks"], overruns=st["overruns"], stale=st["stale_samples"],
                 errors=sum(st.get("device_errors", [])), timeouts=sum(st.get("device_timeouts", [])),
                 scrapes=len(lat), scrape_errors=res.get("errors", 0),
                 scrape_p99_ms=round(lat[int(0.99 * (len(lat) - 1))] * 1e3, 3) if lat else None)
        windows.append(w)
        print(json.dumps(w), flush=True)
    if child is not None:
        rc = child.stop()
        if rc == 0:
            import shutil

            shutil.rmtree(child.workdir, ignore_errors=True)
    else:
        mon.stop()
        rc = None
    if load:
        lst = load.stats()
        load.stop()
    else:
        lst = {}
    first, last = windows[0], windows[-1]
    summary = {"exporter": "bin/gpumon-exporter (child)" if child is not None else "in-process",
               "exporter_exit_status": rc, "minutes": a.minutes, "interval_s": a.interval, "keep_alive": not a.no_keepalive, "windows": len(windows),
               "rss_mb_start": first["rss_mb"], "rss_mb_end": last["rss_mb"],
               "rss_mb_growth_after_first_window": round(last["rss_mb"] - first["rss_mb"], 1),
               "fds_start": first["fds"], "fds_end": last["fds"], "threads_end": last["threads"],
               "ticks": last["ticks"], "overruns": last["overruns"], "device_errors": last["errors"],
               "scrapes": sum(w["scrapes"] for w in windows), "scrape_errors": sum(w["scrape_errors"] for w in windows),
               "scrape_p99_ms_max_window": max(w["scrape_p99_ms"] or 0 for w in windows),
               "load_tflops": round(lst.get("tflops", 0.0), 1), "load_tbps": round(lst.get("tbps", 0.0), 3),
               "baseline_before_start": base}
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
