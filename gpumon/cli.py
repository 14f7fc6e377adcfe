"""``python -m gpumon`` — command line.

    gpumon serve   [--backend amdsmi] [--interval 1] [--listen :9400] ...           run the exporter
    gpumon once    [--format prom|influx|json]                                       one sample to stdout
    gpumon top     [--interval 1] [--url HOST:PORT ... [--ca-file PEM] [--token-file F]]  live console table
    gpumon scrape  URL [-n 1000] [-c 4]                                              scrape-latency probe
    gpumon probe   [--blocks 1024]                                                   run the K1 probe once
    gpumon load    [--kind mixed --seconds 10]                                       synthetic gfx950 load
    gpumon xgmi    [--pairs 0:1,1:0 | --all-pairs] [--seconds 2]                     xGMI link-map validation
    gpumon doctor  [serve flags] [--ondevice-check] [--format text|json]              node prerequisites check

Reference: the agent had no CLI, only ``python3 /gpu.py`` with env vars (Dockerfile:7,
gpu.py:17-26); its display-table formatter (gpu.py:155-168) was dead code — ``gpumon top`` is
that view, implemented.
"""

from __future__ import annotations

import argparse
import json
import logging
import signal
import sys
import threading
import time

from .config import ConfigError, add_cli_args, from_args, redact_url


def _setup_logging(level: str):
    logging.basicConfig(level=getattr(logging, level.upper(), logging.INFO),
                        format="ts=%(asctime)s level=%(levelname)s component=%(name)s msg=%(message)r")


def raise_nofile_limit() -> None:
    """The soft fd limit up to the hard one, as the native binary does (csrc/exporter_main.cpp):
    container runtimes often leave the soft limit at 1024, and the HTTP connection cap is derived
    from it."""
    import resource

    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    if soft != resource.RLIM_INFINITY and (hard == resource.RLIM_INFINITY or soft < hard):
        try:
            resource.setrlimit(resource.RLIMIT_NOFILE, (hard, hard))
        except (ValueError, OSError):
            pass


def cmd_serve(args) -> int:
    from .monitor import GpuMonitor

    cfg = from_args(args).validate()
    _setup_logging(cfg.log_level)
    raise_nofile_limit()
    try:
        mon = GpuMonitor(cfg).start()
    except RuntimeError as e:  # the listen address taken, a mock backend that failed, ...
        print(f"gpumon serve: {e}", file=sys.stderr)
        return 1
    log = logging.getLogger("gpumon")
    log.info("serving %s backend=%s host=%s interval=%.3fs influx=%s control_plane=%s", mon.url, cfg.backend,
             mon.options.host, cfg.interval, redact_url(cfg.influx_url) or "-", mon.control_plane_mode)
    stop = threading.Event()
    for s in (signal.SIGINT, signal.SIGTERM):
        signal.signal(s, lambda *_: stop.set())
    # SIGHUP: re-check the /metrics TLS files now (a rotated certificate is also found within 5 s)
    signal.signal(signal.SIGHUP, lambda *_: mon.ex.reload_tls())
    while not stop.wait(1.0):
        pass
    mon.stop()
    return 0


def cmd_once(args) -> int:
    from .monitor import GpuMonitor

    cfg = from_args(args)
    cfg.interval = 0
    cfg.listen = "127.0.0.1:0"
    _setup_logging(cfg.log_level)
    with GpuMonitor(cfg) as mon:
        time.sleep(0.05)
        mon.step_ondevice()  # make sure the PMC / probe samplers contributed to this sample
        mon.tick()  # second tick: rates populated
        if args.format == "influx":
            sys.stdout.write(mon.ex.influx_text())
        elif args.format == "json":
            json.dump({"devices": mon.ex.statics(), "samples": mon.ex.samples(), "rates": mon.ex.rates(),
                       "pods": mon.ex.pod_rows(), "self": mon.ex.self_stats()}, sys.stdout, indent=1, default=str)
            sys.stdout.write("\n")
        else:
            sys.stdout.write(mon.metrics())
    return 0


def cmd_doctor(args) -> int:
    from . import doctor

    cfg = from_args(args)
    if not getattr(args, "cfgflag__log_level", None):
        cfg.log_level = "error"  # the report is the output
    _setup_logging(cfg.log_level)
    return doctor.main(args, cfg)


def _fmt(v, w, p=0):
    if v is None or v != v:  # None or NaN (not measured)
        return "-".rjust(w)
    return f"{v:{w}.{p}f}"


def render_top(statics, samples, rates, rows, active=None, contexts=None) -> str:
    """Console table (the reference's unused displayfmt columns, gpu.py:156-168, plus MI355X fields).
    `active`: gpu_id -> gpu_active_processes (the sharing state); `contexts`: the exporter's
    /debug/procs view, whose contexts without a row are listed with the reason."""
    from .export.fleet import sharing_label

    lines = []
    hdr = (f"{'GPU':>3} {'UTIL%':>6} {'XCD busy% (0-7)':<32} {'VRAM MiB':>17} {'PWR W':>6} {'HOT C':>6} {'GFX MHz':>8}"
           f" {'PCIe GB/s':>9} {'SHARING':>10}")
    lines.append(hdr)
    for st, sm, rt in zip(statics, samples, rates):
        f = sm["fields"]
        xcd = " ".join(f"{int(x):3d}" if x is not None else "  -" for x in sm["xcd_busy"][:8])
        used = (f["vram_used"] or 0) / 1048576
        tot = (f["vram_total"] or 0) / 1048576
        lines.append(f"{st['gpu_id']:>3} {_fmt(f['gfx_util'], 6)} {xcd:<32} {used:8.0f}/{tot:8.0f} "
                     f"{_fmt(f['power_cur'], 6)} {_fmt(f['temp_hotspot'], 6)} {_fmt(f['gfxclk_cur'], 8)}"
                     f" {_fmt((rt or {}).get('pcie_Bps', float('nan')) / 1e9, 9, 2)}"
                     f" {sharing_label((active or {}).get(str(st['gpu_id']))):>10}")
    lines.append("")
    # BUSY%: share of the interval with the process's waves resident (KFD; the reference copied the
    # device's utilisation onto every process, gpu.py:205); CUs: mean CU-equivalents its waves held;
    # Q: its hardware queues on that GPU (KFD; - where the list is not readable)
    lines.append(f"{'CONTAINER':<13}{'POD':<32}{'NAMESPACE':<14}{'USER':<10}{'PID':>8} {'GPU':>3} {'MEM MiB':>9} "
                 f"{'BUSY%':>6} {'CUs':>6} {'Q':>3}  PROCESS")
    for r in rows:
        lines.append(f"{r['containerid'][:12]:<13}{r['podname'][:31]:<32}{r['namespace'][:13]:<14}{r['user_name'][:9]:<10}"
                     f"{r['pid']:>8} {r['dev']:>3} {r['used_memory_bytes'] / 1048576:9.0f} "
                     f"{_fmt(r['proc_gfx_util'], 6, 1)} {_fmt(r.get('cu_occupancy'), 6, 1)} "
                     f"{r['queues'] if r.get('queues', -1) >= 0 else '-':>3}  {r['procname'][:30]}")
    hidden = [c for c in (contexts or []) if not c.get("row")]
    if hidden:
        # GPU contexts that are not rows: empty (no VRAM, no waves), peer (a multi-GPU process's
        # context on a GPU it does no work on), the exporter's own helper, or not opted in
        lines.append("hidden: " + ", ".join(f"pid {c['pid']} gpu {c['dev']} {c['why']}" for c in hidden[:12])
                     + (f" (+{len(hidden) - 12} more)" if len(hidden) > 12 else ""))
    return "\n".join(lines)


def cmd_top(args) -> int:
    if args.url:
        return _top_remote(args)
    from .monitor import GpuMonitor

    cfg = from_args(args)
    cfg.listen = "127.0.0.1:0"
    with GpuMonitor(cfg) as mon:
        n = 0
        while args.iterations <= 0 or n < args.iterations:
            mon.wait_ticks(1, timeout_s=cfg.interval * 5 + 5)
            from .export import promtext

            fam = promtext.parse(mon.metrics())
            active = {l["gpu_id"]: v for _, l, v in fam.get("gpu_active_processes", {}).get("samples", [])}
            text = render_top(mon.ex.statics(), mon.ex.samples(), mon.ex.rates(), mon.ex.pod_rows(), active,
                              mon.ex.debug_view("/debug/procs"))
            if sys.stdout.isatty():
                sys.stdout.write("\x1b[2J\x1b[H")
            sys.stdout.write(text + "\n")
            sys.stdout.flush()
            n += 1
    return 0


def _top_remote(args) -> int:
    """Fleet view: read running exporters' /metrics instead of opening a GPU (export/fleet.py)."""
    from .export import fleet

    urls = [u if "://" in u else f"http://{u}" for u in args.url]
    urls = [u if u.rstrip("/").endswith("/metrics") else u.rstrip("/") + "/metrics" for u in urls]
    token = ""
    if args.token_file:
        from ._native import core

        err, token, _ = core().read_token_file(args.token_file)  # the first line's token
        if err:
            sys.stderr.write(f"--token-file: {err}\n")
            return 2
    n, rc = 0, 0
    while args.iterations <= 0 or n < args.iterations:
        t0 = time.monotonic()
        frames, errors = fleet.fetch(urls, ca_file=args.ca_file, token=token)
        text = fleet.render(frames, errors)
        if sys.stdout.isatty():
            sys.stdout.write("\x1b[2J\x1b[H")
        sys.stdout.write(text + "\n")
        sys.stdout.flush()
        rc = 1 if errors and not frames else 0
        n += 1
        if args.iterations <= 0 or n < args.iterations:
            interval = float(getattr(args, "cfgflag__interval", None) or 1.0)  # --interval: the refresh period
            time.sleep(max(0.0, interval - (time.monotonic() - t0)))
    return rc


def cmd_scrape(args) -> int:
    from urllib.parse import urlparse

    from ._native import core

    u = urlparse(args.url)
    r = core().scrape_load(u.hostname or "127.0.0.1", u.port or 80, u.path or "/metrics", n_requests=args.n,
                           concurrency=args.c, keep_alive=not args.no_keepalive, gzip=args.gzip)
    lat = sorted(r["latencies_s"])

    def q(p):
        return lat[min(len(lat) - 1, int(p * (len(lat) - 1)))] * 1e3 if lat else float("nan")

    print(json.dumps({"requests": len(lat), "errors": r["errors"], "p50_ms": q(0.5), "p99_ms": q(0.99),
                      "max_ms": lat[-1] * 1e3 if lat else None, "rps": len(lat) / r["wall_s"] if r["wall_s"] else 0,
                      "bytes_per_req": r["bytes"] / max(1, len(lat))}))
    return 0 if r["errors"] == 0 else 1


def cmd_probe(args) -> int:
    from ._native import hip

    H = hip()
    p = H.Probe(args.device, args.blocks, 2, args.spin_ticks)
    slot = p.launch()
    r = p.poll(slot, 5.0)
    if r is None:
        print("probe timed out", file=sys.stderr)
        return 1
    r.pop("records")
    print(json.dumps(r))
    return 0


def cmd_load(args) -> int:
    from .ops.load import SyntheticLoad

    with SyntheticLoad(args.device, args.kind, duty=args.duty, mfma_dtype=args.dtype, period_s=args.period,
                       pcie_direction=args.pcie_direction) as load:
        time.sleep(args.seconds)
        print(json.dumps(load.stats()))
    return 0


def cmd_xgmi(args) -> int:
    """Peer-copy each (src, dst) pair and check that the exporter sees the traffic on the link it
    attributes to dst (validation load for the per-link xGMI fields)."""
    from ._native import core as _core
    from ._native import hip
    from .parallel.xgmi import validate_pair

    n = hip().device_count()  # the peer copies run on the native HIP path (no torch needed)
    if n < 2:
        print(json.dumps({"skipped": f"needs >= 2 GPUs, found {n}"}))
        return 0
    if args.all_pairs:
        pairs = [(a, b) for a in range(n) for b in range(n) if a != b]
    else:
        pairs = [tuple(int(x) for x in p.split(":")) for p in args.pairs.split(",")]
    from .parallel.devmap import hip_bdfs, index_of, match

    bdfs = hip_bdfs(range(n))  # the exporter samples these GPUs, named by PCI address (devmap.py)
    ex = _core().Exporter({"backend": args.backend, "devices": [bdfs[k] for k in range(n)], "serve_http": False,
                           "interval_s": args.interval, "link_every": 1, "processes": False})
    err = ex.start()
    if err:
        print(err, file=sys.stderr)
        return 1
    ok = True
    try:
        idx = index_of(match(bdfs, ex.statics()))
        for src, dst in pairs:
            r = validate_pair(ex, src, dst, seconds=args.seconds, interval=args.interval, index_of=idx)
            ok &= r["peer_matches"]
            print(json.dumps(r), flush=True)
    finally:
        ex.stop()
    return 0 if ok else 1


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="gpumon", description="MI355X Kubernetes GPU telemetry exporter")
    sub = p.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("serve", help="run the exporter")
    add_cli_args(s)
    s.set_defaults(fn=cmd_serve)
    s = sub.add_parser("once", help="take one sample and print it")
    add_cli_args(s)
    s.add_argument("--format", choices=["prom", "influx", "json"], default="prom")
    s.set_defaults(fn=cmd_once)
    s = sub.add_parser("top", help="live console view (local GPUs, or running exporters with --url)")
    add_cli_args(s)
    s.add_argument("--iterations", type=int, default=0)
    s.add_argument("--url", action="append", default=[],
                   help="exporter to read instead of the local GPUs (HOST:PORT or URL; repeat for a fleet view)")
    s.add_argument("--ca-file", default="",
                   help="https:// exporters (tls_cert_file): the PEM CA to verify them with (default: system bundle)")
    s.add_argument("--token-file", default="",
                   help="exporters with http_auth_token_file: the file holding their bearer token")
    s.set_defaults(fn=cmd_top)
    s = sub.add_parser("scrape", help="measure /metrics latency")
    s.add_argument("url")
    s.add_argument("-n", type=int, default=1000)
    s.add_argument("-c", type=int, default=1)
    s.add_argument("--gzip", action="store_true")
    s.add_argument("--no-keepalive", action="store_true")
    s.set_defaults(fn=cmd_scrape)
    s = sub.add_parser("probe", help="run the gfx950 probe kernel once")
    s.add_argument("--device", type=int, default=0)
    s.add_argument("--blocks", type=int, default=1024)
    s.add_argument("--spin-ticks", type=int, default=200)
    s.set_defaults(fn=cmd_probe)
    s = sub.add_parser("load", help="synthetic gfx950 load")
    s.add_argument("--device", type=int, default=0)
    s.add_argument("--kind", choices=["mfma", "hbm", "mixed", "concurrent", "partial", "pcie"], default="mixed")
    s.add_argument("--pcie-direction", choices=["h2d", "d2h", "both"], default="both",
                   help="--kind pcie: pinned host -> device, device -> host, or both at once")
    s.add_argument("--duty", type=float, default=1.0)
    s.add_argument("--period", type=float, default=0.0, help="burst period in s (duty = busy fraction of it)")
    s.add_argument("--seconds", type=float, default=10.0)
    s.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "fp8", "f32", "f64", "i8", "mxfp8", "mxfp4"],
                   help="matrix path of the mfma burn")
    s.set_defaults(fn=cmd_load)
    s = sub.add_parser("doctor", help="check what this node gives the exporter (backend, sysfs, KFD, hostPID, "
                                      "kubelet / CRI sockets, RAS, rt_priority, on-device plugins)")
    add_cli_args(s)
    s.add_argument("--ondevice-check", action="store_true", help="also run the PMC and probe samplers once")
    s.add_argument("--format", choices=["text", "json"], default="text")
    s.set_defaults(fn=cmd_doctor)
    s = sub.add_parser("xgmi", help="validate the per-link xGMI counters with peer copies")
    s.add_argument("--pairs", default="0:1")
    s.add_argument("--all-pairs", action="store_true")
    s.add_argument("--seconds", type=float, default=2.0)
    s.add_argument("--interval", type=float, default=0.1)
    s.add_argument("--backend", default="amdsmi")
    s.set_defaults(fn=cmd_xgmi)
    return p


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    try:
        return args.fn(args)
    except ConfigError as e:
        print(f"config: {e}", file=sys.stderr)
        return 2


if __name__ == "__main__":
    sys.exit(main())
