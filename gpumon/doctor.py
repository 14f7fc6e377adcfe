"""``gpumon doctor``: does this node give the exporter what it needs? (operations runbook)

The reference's only self-check was ``commandexists('docker') and commandexists('nvidia-smi')``
at start-up (/root/reference/gpu.py:28-33,260), printing "Command(s) not found" and exiting.
This runs the exporter's own code paths once and reports, per requirement of
docs/operations.md ("What the DaemonSet needs on an MI355X node"), whether it is met and what is
lost when it is not:

    gpumon doctor [serve flags] [--ondevice-check] [--format text|json]

Exit status 1 when a required check fails (no device backend), 0 otherwise; warnings name the
series that will be missing.
"""

from __future__ import annotations

import json
import os
import re
import sys
import time

OK, WARN, FAIL, SKIP = "ok", "warn", "fail", "skip"


def _gauge(text: str, name: str):
    m = re.search(rf"^{name}(?:{{[^}}]*}})? (\S+)$", text, re.M)
    return float(m.group(1)) if m else None


def _rt_permitted() -> tuple:
    """Whether this process may run SCHED_FIFO threads (rt_priority); restores the policy."""
    if not hasattr(os, "sched_setscheduler"):
        return SKIP, "no sched_setscheduler on this platform"
    old = os.sched_getscheduler(0), os.sched_getparam(0)
    try:
        os.sched_setscheduler(0, os.SCHED_FIFO, os.sched_param(1))
    except PermissionError:
        return WARN, ("SCHED_FIFO not permitted (no CAP_SYS_NICE): rt_priority / http_rt_priority fall back to normal "
                      "scheduling")
    except OSError as e:
        return WARN, f"SCHED_FIFO: {e}"
    finally:
        try:
            os.sched_setscheduler(0, old[0], old[1])
        except OSError:
            pass
    return OK, ("SCHED_FIFO permitted: rt_priority keeps ticks on their deadline, http_rt_priority keeps scrapes "
                "fast on a saturated node")


def fd_table_check(procfs: str = "/proc", pid=None) -> tuple:
    """(status, detail): can this process read another uid's /proc/<pid>/fd table (the /dev/kfd
    ownership check and the fast path's per-process DRM engine time)? Listing the directory needs
    the same uid or CAP_DAC_READ_SEARCH, its links and fdinfo need CAP_SYS_PTRACE
    (tests/test_capabilities.py)."""
    me = os.getuid()
    pids = [str(pid)] if pid is not None else sorted(os.listdir(procfs), key=lambda x: (len(x), x))
    for p in pids:
        if not p.isdigit() or int(p) == os.getpid():
            continue
        try:
            if os.stat(f"{procfs}/{p}").st_uid == me:
                continue
        except OSError:
            continue
        try:
            fds = os.listdir(f"{procfs}/{p}/fd")
        except PermissionError:
            return WARN, (f"pid {p} (uid {os.stat(f'{procfs}/{p}').st_uid}): its fd table cannot be listed (needs "
                          "CAP_DAC_READ_SEARCH): tenants running as another uid get no /dev/kfd check and no DRM "
                          "engine time")
        except OSError:
            continue
        for fd in fds:
            try:
                os.readlink(f"{procfs}/{p}/fd/{fd}")
                return OK, f"another uid's fd table is readable (pid {p})"
            except PermissionError:
                return WARN, (f"pid {p}: fd links unreadable (needs CAP_SYS_PTRACE): no /dev/kfd check and no DRM "
                              "engine time for other uids' tenants")
            except OSError:
                continue
    return SKIP, "no process of another uid with open files to try"


def kfd_queue_check(kfd: str = "/sys/class/kfd/kfd/proc") -> tuple:
    """(status, detail): are KFD's per-process queue lists readable? They decide which GPU contexts of
    a multi-GPU process are peer contexts (no queue there: not a row, whatever their VRAM); without
    them the exporter falls back to the peer_context_max_vram_mib threshold (profiles/r6_kfd_queues.md)."""
    try:
        pids = [e for e in os.listdir(kfd) if e.isdigit()]
    except OSError:
        return SKIP, f"{kfd} not readable"
    if not pids:
        return SKIP, "no KFD process on the node to try"
    readable = queues = 0
    for p in pids:
        try:
            qs = [q for q in os.listdir(f"{kfd}/{p}/queues") if q.isdigit()]
        except OSError:
            continue
        readable += 1
        queues += len(qs)
    if readable == 0:
        return WARN, (f"queues/ of {len(pids)} KFD process(es) unreadable: peer contexts of multi-GPU processes are "
                      "told apart by the VRAM threshold (peer_context_max_vram_mib) instead of their queues")
    return OK, f"queue lists readable for {readable}/{len(pids)} KFD process(es), {queues} queue(s)"


def fd_limit_cap(http_threads: int, limit=None) -> int:
    """The HTTP server's per-loop connection cap for a RLIMIT_NOFILE soft limit (the formula of
    HttpServer::start, csrc/core/http_server.cpp; the running exporter exports the product as
    gpumon_http_max_connections, and a test keeps the two equal)."""
    import resource

    soft = limit if limit is not None else resource.getrlimit(resource.RLIMIT_NOFILE)[0]
    if soft == resource.RLIM_INFINITY:
        return 4096
    usable = soft - 256 if soft > 512 else soft // 2
    return max(8, min(4096, usable // max(1, http_threads)))


def fd_limit_check(http_threads: int, limit=None) -> tuple:
    """A low RLIMIT_NOFILE leaves few scrape connections (256 fds are kept for the sampler). Both
    entry points raise their soft limit to the hard one at startup, so the hard limit is the one
    that counts."""
    import resource

    soft = limit if limit is not None else resource.getrlimit(resource.RLIMIT_NOFILE)[1]
    if soft == resource.RLIM_INFINITY:
        return OK, "RLIMIT_NOFILE unlimited: 4096 connections per HTTP loop"
    cap = fd_limit_cap(http_threads, soft)
    status = OK if cap >= 256 else WARN
    return status, (f"RLIMIT_NOFILE {soft}: {cap} connections per HTTP loop ({http_threads} loop(s))"
                    + ("" if status == OK else ": a connection flood evicts scrapers early; raise the pod's nofile limit"))


def firmware_table_check(path: str, interval_s: float, prewarm_ms: float, seconds: float = 0.25) -> tuple:
    """(status, detail) for one GPU's gpu_metrics file: how often the SMU rewrites it (a new
    firmware_timestamp, v1.8 offset 288; the driver stamps system_clock at every read, so raw bytes
    always differ) against the sampling interval, and what a read costs cold (after 100 ms) vs 3 ms
    after another read -- the gain prewarm_ms buys (profiles/r3_capacity.md)."""
    import struct

    try:
        fd = os.open(path, os.O_RDONLY)
    except OSError as e:
        return WARN, f"{path}: {e.strerror}"
    try:
        b = os.pread(fd, 65536, 0)
        if len(b) < 296 or (b[2], b[3]) != (1, 8):
            return SKIP, f"gpu_metrics v{b[2] if len(b) > 2 else '?'}.{b[3] if len(b) > 3 else '?'}: cadence not decoded"
        last, seen, t_end = struct.unpack_from("<Q", b, 288)[0], 0, time.perf_counter() + seconds
        first_t = last_t = None
        while time.perf_counter() < t_end:
            fw = struct.unpack_from("<Q", os.pread(fd, 65536, 0), 288)[0]
            if fw != last:
                last, seen = fw, seen + 1
                last_t = time.perf_counter()
                first_t = first_t or last_t
        period = (last_t - first_t) / (seen - 1) if seen > 1 else None

        def read_after(gap_s, prefetch):
            lat = []
            for _ in range(5):
                time.sleep(gap_s)
                if prefetch:
                    os.pread(fd, 65536, 0)
                    time.sleep(0.003)
                t0 = time.perf_counter()
                os.pread(fd, 65536, 0)
                lat.append(time.perf_counter() - t0)
            return sorted(lat)[2] * 1e6

        cold, warm = read_after(0.1, False), read_after(0.1, True)
    finally:
        os.close(fd)
    if period is None:
        return WARN, f"the firmware table did not advance in {seconds:.2f} s"
    detail = (f"rewritten every {period * 1e3:.1f} ms ({1 / period:.0f} Hz); a read costs {cold:.0f} us cold, "
              f"{warm:.0f} us 3 ms after another (prewarm_ms {prewarm_ms:g})")
    if 0 < interval_s < period * 0.95:
        return WARN, detail + f": interval {interval_s * 1e3:g} ms is shorter, so some samples repeat a table"
    return OK, detail


def listen_check(listen: str) -> tuple:
    """The configured listen address: parses (the native rule), the families it will serve, and
    whether the port is free (a running exporter on it makes a second one exit EADDRINUSE)."""
    import socket

    from .config import ConfigError, parse_listen

    try:
        host, port = parse_listen(listen)
    except ConfigError as e:
        return (FAIL, str(e))
    v6 = True
    try:
        socket.socket(socket.AF_INET6, socket.SOCK_STREAM).close()
    except OSError:
        v6 = False
    if host in ("", "::"):
        fam = "IPv4 + IPv6 (one dual-stack [::] socket)" if v6 else (
            "IPv4 only: no IPv6 in this network namespace" + (" -- [::] will fail" if host == "::" else ""))
    else:
        fam = "IPv6 only" if ":" in host else "IPv4 only" if host.replace(".", "").isdigit() or host == "0.0.0.0" else host
    if port == 0:
        return (OK, f"{listen}: {fam}, ephemeral port")
    fam_bind = socket.AF_INET6 if (v6 and host in ("", "::")) or ":" in host else socket.AF_INET
    s = socket.socket(fam_bind, socket.SOCK_STREAM)
    try:
        if fam_bind == socket.AF_INET6 and host in ("", "::"):
            s.setsockopt(socket.IPPROTO_IPV6, socket.IPV6_V6ONLY, 0)
        s.bind((host or ("::" if fam_bind == socket.AF_INET6 else "0.0.0.0"), port))
        free = True
    except OSError as e:
        free = e.errno != 98  # EADDRINUSE
        if free:
            return (WARN, f"{listen}: {fam}; cannot bind: {e.strerror}")
    finally:
        s.close()
    return (OK, f"{listen}: {fam}, port {port} free") if free else (
        WARN, f"{listen}: {fam}; port {port} is in use (an exporter already running here? a second one exits "
              "with EADDRINUSE)")


def influx_check(cfg) -> tuple:
    """The Influx compat push: the startup check both entry points run (scheme, host, TLS files,
    libssl), then one GET /ping on the same host over the same transport (TLS verified as the
    push will be): reachability without writing anything."""
    from ._native import core as _core
    from .config import redact_url

    c = _core()
    err = c.check_push_config(cfg.influx_url, cfg.influx_token, cfg.influx_ca_file, bool(cfg.influx_tls_insecure),
                              cfg.influx_client_cert, cfg.influx_client_key)
    if err:
        return (FAIL, err + ": the exporter refuses to start with it")
    u = c.parse_url(cfg.influx_url)
    host = f"[{u['host']}]" if ":" in u["host"] else u["host"]
    ping = f"{'https' if u['tls'] else 'http'}://{host}:{u['port']}/ping"
    st, _, perr = c.http_request("GET", ping, "", "", 3.0, cfg.influx_ca_file, bool(cfg.influx_tls_insecure))
    what = redact_url(cfg.influx_url) + (" (TLS, certificate verified)" if u["tls"] and not cfg.influx_tls_insecure
                                         else " (TLS, NOT verified)" if u["tls"] else "")
    if st in (200, 204):
        return (OK, f"{what}: /ping answered {st}")
    return (WARN, f"{what}: /ping " + (f"answered HTTP {st}" if st > 0 else f"failed: {perr}")
            + "; the push will retry with backoff (gpumon_influx_up 0 until it succeeds)")


def serve_tls_check(cfg, now=None) -> tuple:
    """/metrics over HTTPS: the certificate, key and client CA load (the startup check), and the
    certificate's remaining validity (the GpumonMetricsCertificateExpiring alert fires under 7 days)."""
    import time

    from ._native import core as _core

    err, not_after = _core().serve_tls_not_after(cfg.tls_cert_file, cfg.tls_key_file, cfg.tls_client_ca_file)
    if err:
        return (FAIL, err + ": the exporter refuses to start with it")
    mtls = ", mutual TLS" if cfg.tls_client_ca_file else ""
    if not not_after:
        return (OK, f"{cfg.tls_cert_file}{mtls}: loads (expiry unknown)")
    days = (not_after - (now if now is not None else time.time())) / 86400
    when = time.strftime("%Y-%m-%d", time.gmtime(not_after))
    if days < 0:
        return (FAIL, f"{cfg.tls_cert_file}{mtls}: EXPIRED on {when}: every verifying scraper is refused")
    if days < 7:
        return (WARN, f"{cfg.tls_cert_file}{mtls}: expires {when} ({days:.1f} days): renew it (rotation is picked up "
                      "without a restart)")
    return (OK, f"{cfg.tls_cert_file}{mtls}: valid until {when} ({days:.0f} days)")


def auth_token_check(cfg) -> tuple:
    """/metrics behind a bearer token: the file holds a usable token (the startup check)."""
    from ._native import core as _core

    err, _, tokens = _core().read_token_file(cfg.http_auth_token_file)
    if err:
        return (FAIL, err + ": the exporter refuses to start with it")
    import os
    import stat

    short = min(len(t) for t in tokens)
    which = f"{len(tokens)} tokens accepted (a rotation in progress?)" if len(tokens) > 1 else "1 token"
    if os.stat(cfg.http_auth_token_file).st_mode & stat.S_IROTH:
        return (WARN, f"{cfg.http_auth_token_file}: {which}, but the file is readable by every user on the node: "
                      "mode 0400 / 0440 (the overlay's Secret uses defaultMode 0400)")
    if short < 16:
        return (WARN, f"{cfg.http_auth_token_file}: {which}, one of {short} characters: use 16 or more random "
                      "characters")
    return (OK, f"{cfg.http_auth_token_file}: {which}; /metrics answers 401 without it")


def run(cfg, ondevice_check: bool = False, wait_s: float = 3.0) -> list:
    """[(check, status, detail)] for the node this runs on, with the exporter configured as `cfg`."""
    from .monitor import GpuMonitor

    out = []
    interval_s = cfg.interval  # as configured (the checks below tick by hand)
    out.append(("listen address",) + listen_check(cfg.listen))
    if cfg.tls_cert_file or cfg.tls_key_file or cfg.tls_client_ca_file:
        out.append(("/metrics TLS certificate",) + serve_tls_check(cfg))
        cfg.tls_cert_file = cfg.tls_key_file = cfg.tls_client_ca_file = ""  # the checks below serve plain
    if cfg.http_auth_token_file:
        out.append(("/metrics bearer token",) + auth_token_check(cfg))
        cfg.http_auth_token_file = ""  # ... and scrape without a token
    if cfg.influx_url:
        out.append(("Influx push",) + influx_check(cfg))
        cfg.influx_url = ""  # checked above; the checks below do not push
    cfg.interval = 0
    cfg.listen = "127.0.0.1:0"
    cfg.enable_pmc = cfg.enable_probe = False  # the on-device check below runs them explicitly
    mon = GpuMonitor(cfg).start()
    try:
        st = mon.ex.self_stats()
        if mon.start_error or not st.get("backend_up"):
            out.append(("device backend", FAIL, mon.start_error or "backend down"))
            return out
        statics = mon.ex.statics()
        archs = sorted({s.get("gfx_target", "?") for s in statics})
        out.append(("device backend", OK, f"{st.get('backend')} {st.get('backend_version', '')}".strip()
                     + f": {len(statics)} GPU(s), {', '.join(archs)}"))
        if any(a != "gfx950" for a in archs):
            out.append(("gfx950", WARN, f"targets {archs}: the probe / load kernels are built for gfx950 only"))
        fp = st.get("fast_path_devices", 0)
        if fp < 0:
            out.append(("sysfs fast path", SKIP, f"not applicable to the {st.get('backend')} backend"))
        else:
            out.append(("sysfs fast path", OK if fp == len(statics) else WARN,
                        f"{fp}/{len(statics)} GPU(s) ({st.get('fast_path_status', '')})"
                        + ("" if fp == len(statics) else ": the rest goes through libamd_smi (about 2x the tick time)")))
        if statics and statics[0].get("bdf") and os.path.exists(f"/sys/bus/pci/devices/{statics[0]['bdf']}/gpu_metrics"):
            out.append(("firmware table",) + firmware_table_check(
                f"/sys/bus/pci/devices/{statics[0]['bdf']}/gpu_metrics", interval_s, cfg.prewarm_ms))
        else:
            out.append(("firmware table", SKIP, "no gpu_metrics file for the first GPU"))
        kfd = "/sys/class/kfd/kfd/proc"
        if os.access(kfd, os.R_OK):
            try:
                n_kfd = sum(1 for e in os.listdir(kfd) if e.isdigit())
            except OSError:
                n_kfd = -1
            out.append(("KFD process table", OK, f"{kfd} readable, {n_kfd} KFD process(es) on the host (every GPU; "
                                                 "each tick reads the ones on the sampled GPUs)"))
        else:
            out.append(("KFD process table", WARN,
                        f"{kfd} not readable: no per-process rows (pod_gpu_*), no occupancy / busy %"))
        out.append(("KFD queue lists",) + kfd_queue_check(kfd))
        try:
            init = open("/proc/1/comm").read().strip()
        except OSError:
            init = "?"
        host_pid = init in ("systemd", "init")
        out.append(("host PID namespace", OK if host_pid else WARN,
                    f"PID 1 is {init}" + ("" if host_pid else ": not the host's PID namespace; KFD reports host "
                                          "PIDs, so pod attribution needs hostPID: true")))
        ras = [s for s in statics if s.get("bdf") and os.path.isdir(f"/sys/bus/pci/devices/{s['bdf']}/ras")]
        out.append(("RAS / ECC files", OK if ras else WARN,
                    f"ras/ readable on {len(ras)}/{len(statics)} GPU(s)" if ras
                    else "no ras/ directory: ECC from libamd_smi per block, no poison / fatal events"))
        # control plane: the native pollers run at start; give them a moment to report
        deadline = time.time() + wait_s
        text = mon.metrics()
        while time.time() < deadline and (_gauge(text, "gpumon_podresources_up") is None
                                          or _gauge(text, "gpumon_cri_up") is None):
            time.sleep(0.2)
            mon.tick()
            text = mon.metrics()
        for name, series, sock, lost, status in (
                ("kubelet PodResources", "gpumon_podresources", cfg.pod_resources_socket,
                 "no idle-allocation rows, no allocated / in-use GPU counts", "grpc_status"),
                ("CRI runtime", "gpumon_cri", cfg.cri_socket or "(autodetect)",
                 "pod names from /proc fallbacks only (HOSTNAME, service-account namespace)", "grpc_status"),
                ("Docker Engine", "gpumon_docker", cfg.docker_socket or "(off: docker_socket not set)",
                 "container names / labels from CRI or /proc fallbacks only", "http_status")):
            up = _gauge(text, f"{series}_up")
            code = _gauge(text, f"{series}_{status}")
            if up is None:
                out.append((name, SKIP, f"{sock}: not polled (control plane off or no socket)"))
            elif up >= 1:
                out.append((name, OK, f"{sock}: answering"))
            else:
                code_s = "-" if code is None else int(code)
                out.append((name, WARN, f"{sock}: down ({status.replace('_', '-')} {code_s}): {lost}"))
        # socket-free metadata (non-root deployments): the kubelet's log tree / device checkpoint
        for name, src, path, lost in (
                ("kubelet log tree", "pod_logs", cfg.pod_log_root,
                 "containers the CRI source does not name stay at their /proc fallbacks"),
                ("device-plugin checkpoint", "device_checkpoint", cfg.device_checkpoint,
                 "no idle-allocation rows without PodResources (the file is root 0600 by default)")):
            if not path:
                out.append((name, SKIP, f"off ({src.replace('pod_logs', 'pod_log_root')} not set)"))
                continue
            m = re.search(r'^gpumon_kubelet_files_up\{[^}]*source="' + src + r'"[^}]*\} (\S+)$', text, re.M)
            up = float(m.group(1)) if m else None
            out.append((name, OK if up == 1 else WARN, f"{path}: readable" if up == 1 else f"{path}: unreadable: {lost}"))
        out.append(("other uids' fd tables",) + fd_table_check())
        out.append(("file descriptor limit",) + fd_limit_check(int(getattr(cfg, "http_threads", 2) or 2)))
        out.append(("rt_priority / http_rt_priority",) + _rt_permitted())
        # on-device samplers: the helper and plugins must exist; --ondevice-check runs them once
        from ._native import core as _core

        core = _core()
        plugin_dir = cfg.plugin_dir or os.environ.get("GPUMON_PLUGIN_DIR") or os.path.join(
            os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib")
        files = ["gpumon-ondevice-helper", "libgpumon_pmc.so", "libgpumon_probe.so"]
        missing = [f for f in files if not os.path.exists(os.path.join(plugin_dir, f))]
        out.append(("on-device plugins", OK if not missing else WARN,
                    f"{plugin_dir}: " + ("helper + PMC + probe present" if not missing
                                         else f"missing {', '.join(missing)}: enable_pmc / enable_probe will refuse "
                                              "to start")))
        if ondevice_check and not missing:
            od = core.OnDevice(mon.ex, {"plugin_dir": plugin_dir, "pmc": True, "probe": True, "pmc_every_s": 60.0,
                                        "probe_every_s": 60.0, "pmc_mode": "continuous", "ondevice_isolate": True})
            try:
                od.start()
                od.step()
                time.sleep(0.2)
                od.step()
                s = od.stats()
                mon.tick()
                text = mon.metrics()
                pmc_up = _gauge(text, "gpumon_pmc_up")
                out.append(("PMC device counting", OK if pmc_up == 1 else WARN,
                            f"{s['pmc_agents']} agent(s), pmc_up {pmc_up}, errors {s['pmc_errors']}"
                            + ("" if pmc_up == 1 else ": another profiler may hold the counters")))
                out.append(("K1 probe", OK if s["probe_done"] > 0 else WARN,
                            f"{s['probe_devices']} device(s), {s['probe_done']} completed, "
                            f"{s['probe_timeouts']} timeouts"))
                rss = _gauge(text, "gpumon_ondevice_helper_resident_memory_bytes")
                model = _gauge(text, "gpumon_ondevice_helper_memory_model_bytes")
                if rss:
                    over = bool(model) and rss > 1.2 * model
                    out.append(("on-device helper memory", WARN if over else OK,
                                f"{rss / 2 ** 20:.0f} MiB resident"
                                + (f", model {model / 2 ** 20:.0f} MiB for these samplers" if model else "")
                                + (": above the model, raise the overlay's memory limit" if over else
                                   " (the overlays are sized by the model)")))
            except RuntimeError as e:
                out.append(("on-device samplers", FAIL, str(e)))
            finally:
                od.stop()
    finally:
        mon.stop()
    return out


def main(args, cfg) -> int:
    checks = run(cfg, ondevice_check=args.ondevice_check)
    if args.format == "json":
        json.dump([{"check": c, "status": s, "detail": d} for c, s, d in checks], sys.stdout, indent=1)
        sys.stdout.write("\n")
    else:
        for c, s, d in checks:
            sys.stdout.write(f"[{s.upper():>4}] {c:<24} {d}\n")
    return 1 if any(s == FAIL for _, s, _ in checks) else 0
