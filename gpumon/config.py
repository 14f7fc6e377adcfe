"""Typed configuration: defaults < YAML file < environment < CLI flags.

Reference configuration (/root/reference/gpu.py:17-26, gpu_monitor.yaml:29-37):
  * ``NODE_NAME``    — node name tag (fieldRef spec.nodeName); fallback ``"no_name"`` (gpu.py:23-24).
    The reference re-reads the env inside main() so its fallback never reached the emitted lines
    (quirk Q1); here the resolved value is used everywhere, falling back to the hostname.
  * ``INFLUXDB_URL`` — InfluxDB write endpoint; default hard-coded in gpu.py:18,26.
    Here: when set, the Influx compat push is enabled (batched, one POST per tick).
  * sampling interval hard-coded to 10 s (gpu.py:263) -> ``interval`` (default 1 s).
  * opt-in docker label mlgpu=mlgpu hard-coded (gpu.py:186-188) -> ``opt_in_label`` (default off;
    ``--compat`` sets ``mlgpu=mlgpu``).
  * pod-name prefix ``turing-gpu-notebook-`` hard-coded (gpu.py:196,230) -> ``user_prefix``.
"""

from __future__ import annotations

import argparse
import dataclasses
import os
import socket
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml

REFERENCE_DEFAULT_INFLUX = "http://10.0.4.235:9000/write?db=gpu_process"  # gpu.py:18 (not used unless --compat)


@dataclass
class Config:
    # device backend
    backend: str = "auto"                 # auto | amdsmi | rocm_smi | mock[:k=v,...]
    amdsmi_lib: str = ""
    rocm_smi_lib: str = ""                # librocm_smi64 override (rocm_smi backend / auto fallback)
    fast_path: bool = True                # amdsmi: hot per-tick reads straight from sysfs/KFD
    sysfs_root: str = "/sys"
    devices: List[str] = field(default_factory=list)  # hip ids ("3") and / or PCI BDFs ("0000:75:00.0")
    interval: float = 1.0                 # seconds; 0.1 = 10 Hz stress config
    processes: bool = True
    link_every: int = 600                 # ticks between link-metrics refreshes (+ whenever a link's state changes)
    ras_every: int = 5                    # ticks per full RAS / ECC pass (0 = off)
    ras_slices: int = 1                   # the pass read in this many slices on consecutive ticks (1..ras_every)
    ras_async: bool = True                # device workers read RAS after publishing a tick (next tick carries it)
    hide_empty_contexts: bool = True      # no pod_gpu row for a GPU context with no VRAM and no waves
    mfma_exclusive_window_s: float = 5.0  # pod MFMA util only when no other process had waves in the last 5 ticks and this many seconds
    peer_context_max_vram_mib: float = 512.0  # a multi-GPU process's context on a GPU it does not work on (<= this VRAM, no waves, a workload on another GPU): no row (0 = off)
    occ_samples: int = 20                 # KFD cu_occupancy reads per process per tick (device workers; 1 = the tick's own)
    prewarm_ms: float = 3.0               # device workers wake the firmware-table path this long before each tick (0 = off)
    stale_hold_s: float = 0.1             # a repeated firmware table keeps the last rates only while it is this old (then: invalid)
    sample_threads: int = -1              # -1 = one worker per GPU (parallel + watchdog); 0 = sequential
    rt_priority: int = 0                  # SCHED_FIFO priority of the sampler + device workers (needs CAP_SYS_NICE)
    device_timeout_s: float = 2.0         # a device call still running after this is exported as hung
    reinit_after: int = 5                 # ticks with every GPU failing before the backend is re-initialised
    init_retry_s: float = 5.0             # backoff between backend init attempts
    health_stale_s: float = 0.0           # /healthz 503 after this long without a tick (0 = max(3*interval, 10 s))
    # exposition
    listen: str = ":9400"                 # host:port | [v6]:port | :port (every address, dual-stack; IPv4 if no IPv6)
    http_threads: int = 2
    http_rt_priority: int = 0             # SCHED_FIFO HTTP loops (CAP_SYS_NICE), each capped at http_rt_budget of a CPU
    http_rt_budget: float = 0.2           # share of a CPU per 100 ms an RT HTTP loop may use before it is demoted
    tls_cert_file: str = ""               # /metrics over HTTPS: PEM certificate chain (with tls_key_file)
    tls_key_file: str = ""                # ... its PEM private key
    tls_client_ca_file: str = ""          # ... mutual TLS: scrapers must present a certificate signed by this CA
    http_auth_token_file: str = ""        # /metrics needs "Authorization: Bearer <the file's token>" (health endpoints stay open)
    host: str = ""
    gzip: bool = True
    compat_families: bool = True
    extended_families: bool = True
    metrics_include: List[str] = field(default_factory=list)  # serve only families matching these globs (e.g. node_gpu_*)
    metrics_exclude: List[str] = field(default_factory=list)  # drop families matching these globs (e.g. gpu_xcd_*); Influx unfiltered
    # influx compat push
    influx_url: str = ""                  # http(s)://[user:password@]host[:port]/path?query; checked at startup (exit 2 if unusable)
    influx_token: str = ""                # InfluxDB 2.x/3.x API token (env INFLUXDB_TOKEN, from a Secret); 1.x: user:password@ in the URL
    influx_extended: bool = False
    influx_schema: int = 2019             # 2019 = gpu.py layout; 2018 = img/influxdb.png pod_gpu layout
    influx_every: int = 1
    influx_gzip: bool = False             # gzip each push (Content-Encoding: gzip): 7-8x fewer bytes for 8 GPUs
    influx_ca_file: str = ""              # https:// push: PEM CA bundle replacing the system one
    influx_tls_insecure: bool = False     # https:// push WITHOUT certificate / host-name checks (opt-in, testing)
    influx_client_cert: str = ""          # https:// push: PEM client chain for mutual TLS
    influx_client_key: str = ""           # ... and its key (default: in the chain file)
    # attribution
    procfs_root: str = "/proc"
    opt_in_label: str = ""
    user_label: str = ""
    user_regex: str = ""
    # pod / container label keys copied onto pod_gpu_* series as label_<key> (kube-state-metrics style)
    pod_label_allowlist: List[str] = field(default_factory=list)
    user_prefix: str = "turing-gpu-notebook-"
    compat_user_rule: bool = True
    procfs_env_fallback: bool = True
    include_host_processes: bool = True
    # control plane (k8s)
    control_plane: str = "native"         # native (C++ grpc_lite CRI / PodResources / Docker pollers) | off
    cri_socket: str = ""                  # e.g. unix:///run/containerd/containerd.sock ; "" = autodetect ; none = off
    pod_resources_socket: str = "/var/lib/kubelet/pod-resources/kubelet.sock"
    docker_socket: str = ""               # plain-Docker nodes (native plane): Docker Engine container names + labels; opt-in, e.g. /var/run/docker.sock
    # socket-free metadata for a non-root exporter (csrc/core/kubelet_files.h): the kubelet's log tree
    # (containers/ + pods/ under this root) and device-plugin checkpoint; "" = off
    pod_log_root: str = ""                # e.g. /var/log
    device_checkpoint: str = ""           # e.g. /var/lib/kubelet/device-plugins/kubelet_internal_checkpoint
    resource_names: List[str] = field(default_factory=lambda: ["amd.com/gpu"])
    # DRA drivers whose claimed devices count as GPU allocations (kubelet PodResources dynamic_resources)
    dra_drivers: List[str] = field(default_factory=lambda: ["gpu.amd.com"])
    metadata_refresh: float = 10.0
    # on-device probe / PMC
    enable_probe: bool = False
    probe_every: int = 1
    enable_pmc: bool = False
    plugin_dir: str = ""                  # "" = <tree>/lib or $GPUMON_PLUGIN_DIR
    roctx: bool = False                   # ROCTx ranges around sampler phases (rocprofv3 --marker-trace)
    # the counters the PMC derivation needs (csrc/core/ondevice.cpp; 8 SQ + 2 GRBM slots: one counting pass on gfx950):
    # MFMA busy + MFMA MOPS per operand type; no per-wave SQ counters (they count only the profiling
    # process's own waves, profiles/r1_pmc_cross_process.md)
    # continuous: counting contexts run all the time, read without a stop (100 % coverage);
    # window: start -> pmc_window -> stop per period (the r1 sampler)
    pmc_mode: str = "continuous"
    # the counting contexts in a helper process frozen between reads (rocprofiler-sdk leaves an HSA
    # thread polling a full core in the process that owns them, profiles/r2_footprint.md)
    ondevice_isolate: bool = True
    helper_retry: float = 10.0            # seconds before a dead helper is respawned (doubling while it keeps dying)
    pmc_counters: List[str] = field(default_factory=lambda: (
        ["SQ_VALU_MFMA_BUSY_CYCLES"] + ["SQ_INSTS_VALU_MFMA_MOPS_" + d for d in
                                        ("BF16", "F16", "F8", "F6F4", "F32", "F64", "I8")]
        + ["GRBM_GUI_ACTIVE", "GRBM_COUNT"]))
    # rates calibration
    activity_acc_scale: float = 1.0
    xgmi_kb_bytes: float = 1024.0
    log_level: str = "info"

    # ------------------------------------------------------------------ helpers
    @property
    def listen_addr(self) -> str:
        """Host part of `listen` ("" = every address, dual-stack): the native parse_listen rule."""
        return parse_listen(self.listen)[0]

    @property
    def port(self) -> int:
        return parse_listen(self.listen)[1]

    def resolved_host(self) -> str:
        return self.host or os.environ.get("NODE_NAME") or socket.gethostname() or "no_name"

    def to_core(self) -> Dict[str, Any]:
        """Dict consumed by gpumon._core.Exporter."""
        return {
            "backend": self.backend,
            "amdsmi_lib": self.amdsmi_lib,
            "rocm_smi_lib": self.rocm_smi_lib,
            "fast_path": self.fast_path,
            "sysfs_root": self.sysfs_root,
            "devices": _device_ids(self.devices),
            "interval_s": float(self.interval),
            "processes": self.processes,
            "link_every": int(self.link_every),
            "ras_every": int(self.ras_every),
            "ras_slices": int(self.ras_slices),
            "ras_async": bool(self.ras_async),
            "occ_samples": int(self.occ_samples),
            "prewarm_ms": float(self.prewarm_ms),
            "stale_hold_s": float(self.stale_hold_s),
            "hide_empty_contexts": bool(self.hide_empty_contexts),
            "mfma_exclusive_window_s": float(self.mfma_exclusive_window_s),
            "peer_context_max_vram_mib": float(self.peer_context_max_vram_mib),
            "sample_threads": int(self.sample_threads),
            "rt_priority": int(self.rt_priority),
            "device_timeout_s": float(self.device_timeout_s),
            "reinit_after": int(self.reinit_after),
            "init_retry_s": float(self.init_retry_s),
            "health_stale_s": float(self.health_stale_s),
            "listen_addr": self.listen_addr,
            "port": self.port,
            "http_threads": int(self.http_threads),
            "http_rt_priority": int(self.http_rt_priority),
            "http_rt_budget": float(self.http_rt_budget),
            "tls_cert_file": self.tls_cert_file,
            "tls_key_file": self.tls_key_file,
            "tls_client_ca_file": self.tls_client_ca_file,
            "http_auth_token_file": self.http_auth_token_file,
            "host": self.resolved_host(),
            "gzip": self.gzip,
            "roctx": self.roctx,
            "compat_families": self.compat_families,
            "extended_families": self.extended_families,
            "metrics_include": list(self.metrics_include),
            "metrics_exclude": list(self.metrics_exclude),
            "influx_url": self.influx_url,
            "influx_token": self.influx_token,
            "influx_extended": self.influx_extended,
            "influx_schema": int(self.influx_schema),
            "influx_every": int(self.influx_every),
            "influx_gzip": bool(self.influx_gzip),
            "influx_ca_file": self.influx_ca_file,
            "influx_tls_insecure": bool(self.influx_tls_insecure),
            "influx_client_cert": self.influx_client_cert,
            "influx_client_key": self.influx_client_key,
            "procfs_root": self.procfs_root,
            "opt_in": self.opt_in_label,
            "user_label": self.user_label,
            "user_regex": self.user_regex,
            "label_allowlist": list(self.pod_label_allowlist),
            "user_prefix": self.user_prefix,
            "compat_user_rule": self.compat_user_rule,
            "procfs_env_fallback": self.procfs_env_fallback,
            "include_host_processes": self.include_host_processes,
            "activity_acc_scale": float(self.activity_acc_scale),
            "xgmi_kb_bytes": float(self.xgmi_kb_bytes),
            "version": _version(),
        }

    def validate(self) -> "Config":
        """Configuration-time checks the exporter would otherwise only hit while running. The Influx
        push: the same native check bin/gpumon-exporter runs before it starts (csrc/core/tls.h
        check_push_config) -- scheme, host, port, token, and for https libssl plus readable CA /
        client files. Raises ConfigError naming the problem."""
        if self.influx_url:
            from ._native import core

            err = core().check_push_config(self.influx_url, self.influx_token, self.influx_ca_file,
                                           bool(self.influx_tls_insecure), self.influx_client_cert,
                                           self.influx_client_key)
            if err:
                raise ConfigError(err)
        if self.tls_cert_file or self.tls_key_file or self.tls_client_ca_file:
            from ._native import core

            err = core().check_serve_tls(self.tls_cert_file, self.tls_key_file, self.tls_client_ca_file)
            if err:
                raise ConfigError(err)
        if self.http_auth_token_file:
            from ._native import core

            err = core().check_auth_token_file(self.http_auth_token_file)
            if err:
                raise ConfigError("http_auth_token_file: " + err)
        try:
            _device_ids(self.devices)
        except ValueError as e:
            raise ConfigError(str(e)) from None
        parse_listen(self.listen)
        return self

    # ------------------------------------------------------------------ sources
    def apply_dict(self, d: Dict[str, Any]) -> "Config":
        names = {f.name: f for f in dataclasses.fields(self)}
        for k, v in (d or {}).items():
            key = k.replace("-", "_")
            if key in _RETIRED:
                continue  # accepted, no effect (see _RETIRED)
            if key not in names:
                raise ValueError(f"unknown config key: {k}")
            setattr(self, key, _coerce(names[key], v))
        return self

    def apply_env(self, env: Optional[Dict[str, str]] = None) -> "Config":
        env = os.environ if env is None else env
        if env.get("NODE_NAME"):
            self.host = env["NODE_NAME"]
        if env.get("INFLUXDB_URL"):
            self.influx_url = env["INFLUXDB_URL"]
        if env.get("INFLUXDB_TOKEN"):
            self.influx_token = env["INFLUXDB_TOKEN"]
        names = {f.name: f for f in dataclasses.fields(self)}
        for k, v in env.items():
            if k.startswith("GPUMON_") and k != "GPUMON_CONFIG" and k != "GPUMON_AMDSMI_LIB":
                key = k[len("GPUMON_"):].lower()
                if key in names:
                    setattr(self, key, _coerce(names[key], v))
        return self


class ConfigError(ValueError):
    """A configuration the exporter cannot run with (the CLI exits 2 with the message)."""


# Keys of earlier releases that selected the Python test oracles (now under tests/oracles, not
# shipped): a config file that still names them keeps working, with the native path.
_RETIRED = {"ondevice"}


def parse_listen(listen: str):
    """`listen` -> (host, port), the rule of the native parse_listen (csrc/core/http_server.cpp), which
    tests/test_native_config.py checks this against: "host:port", "[v6]:port", ":port", "*:port" or
    "port"; host "" = every address (one dual-stack [::] socket, 0.0.0.0 where the kernel has no
    IPv6). Raises ConfigError for anything else."""
    import ipaddress

    s = str(listen).strip()
    if not s:
        raise ConfigError("empty listen address")
    if s.startswith("["):
        rb = s.find("]")
        if rb < 0 or rb + 1 >= len(s) or s[rb + 1] != ":":
            raise ConfigError(f"listen '{s}': expected [v6]:port")
        host, port = s[1:rb], s[rb + 2:]
        try:
            ipaddress.IPv6Address(host)
        except ValueError:
            raise ConfigError(f"listen '{s}': '{host}' is not an IPv6 address") from None
    elif s.isdigit():
        host, port = "", s
    else:
        if ":" not in s:
            raise ConfigError(f"listen '{s}': expected host:port")
        host, port = s.rsplit(":", 1)
        if ":" in host:
            raise ConfigError(f"listen '{s}': an IPv6 address needs brackets ([v6]:port)")
        if host == "*":
            host = ""
    if not port or len(port) > 5 or not port.isdigit() or int(port) > 65535:
        raise ConfigError(f"listen '{s}': bad port '{port}'")
    return host, int(port)


def redact_url(url: str) -> str:
    """`user:password@` userinfo with the password masked (same rule as the native redact_url in
    csrc/core/http_client.cpp): INFLUXDB_URL may carry 1.x credentials and is logged at startup."""
    scheme = url.find("://")
    start = 0 if scheme < 0 else scheme + 3
    ends = [i for i in (url.find("/", start), url.find("?", start)) if i >= 0]
    end = min(ends) if ends else len(url)
    at = url.rfind("@", 0, end + 1 if ends else len(url))
    if at < start:
        return url
    colon = url.find(":", start)
    if colon < 0 or colon > at:
        return url
    return url[:colon + 1] + "***" + url[at:]


def _device_ids(devices) -> List[str]:
    """`devices` entries as the native filter takes them: a hip id ("3") or a PCI BDF; anything else
    is a configuration error here (the native parser refuses it the same way, csrc/core/options.cpp)."""
    from .parallel.devmap import normalize_bdf

    out = []
    for x in devices:
        s = str(x).strip()
        b = normalize_bdf(s)
        if b:
            out.append(b)
        elif s.isdigit():
            out.append(str(int(s)))
        else:
            raise ValueError(f"devices: {x!r} is neither a hip id nor a PCI BDF")
    return out


def _version() -> str:
    from . import __version__

    return __version__


def _coerce(f: dataclasses.Field, v: Any) -> Any:
    t = f.type if isinstance(f.type, str) else getattr(f.type, "__name__", str(f.type))
    if v is None:
        return v
    if t in ("bool",):
        if isinstance(v, bool):
            return v
        return str(v).strip().lower() in ("1", "true", "yes", "on")
    if t in ("int",):
        return int(v)
    if t in ("float",):
        return float(v)
    if t.startswith("List[int]"):
        if isinstance(v, str):
            return [int(x) for x in v.split(",") if x.strip()]
        return [int(x) for x in v]
    if t.startswith("List[str]"):
        if isinstance(v, str):
            return [x.strip() for x in v.split(",") if x.strip()]
        return [str(x) for x in v]
    return str(v)


def load_yaml(path: str) -> Dict[str, Any]:
    with open(path, "r", encoding="utf-8") as fh:
        data = yaml.safe_load(fh) or {}
    if not isinstance(data, dict):
        raise ValueError(f"{path}: top level must be a mapping")
    return data.get("gpumon", data)


def add_cli_args(p: argparse.ArgumentParser) -> None:
    d = Config()
    p.add_argument("--config", default=os.environ.get("GPUMON_CONFIG", ""), help="YAML config file")
    p.add_argument("--backend", help=f"amdsmi | rocm_smi | mock[:gpus=N,...] | auto (default {d.backend}; "
                   "auto = amdsmi, falling back to rocm_smi)")
    p.add_argument("--devices", help="comma-separated hip ids and / or PCI BDFs to monitor (default all)")
    p.add_argument("--interval", type=float, help=f"sampling interval seconds (default {d.interval})")
    p.add_argument("--listen", help=f"HOST:PORT, [V6]:PORT or :PORT for /metrics (default {d.listen}: every "
                   "address, IPv4 and IPv6)")
    p.add_argument("--host", help="node name label (default $NODE_NAME, then hostname)")
    p.add_argument("--influx-url", dest="influx_url", help="enable InfluxDB line-protocol push (default $INFLUXDB_URL)")
    p.add_argument("--influx-extended", dest="influx_extended", action="store_true", default=None)
    p.add_argument("--influx-gzip", dest="influx_gzip", action="store_true", default=None,
                   help="gzip each Influx push (Content-Encoding: gzip; InfluxDB 1.x / 2.x / 3.x accept it)")
    p.add_argument("--influx-ca-file", dest="influx_ca_file", help="PEM CA bundle for an https:// INFLUXDB_URL "
                   "(default: the system bundle)")
    p.add_argument("--influx-tls-insecure", dest="influx_tls_insecure", action="store_true", default=None,
                   help="do NOT verify the InfluxDB server's certificate (testing only)")
    p.add_argument("--influx-client-cert", dest="influx_client_cert", help="PEM client certificate (mutual TLS)")
    p.add_argument("--influx-client-key", dest="influx_client_key", help="PEM client key (mutual TLS)")
    p.add_argument("--influx-schema", dest="influx_schema", type=int, choices=[2018, 2019],
                   help="pod_gpu line layout: 2019 (gpu.py, default) or 2018 (img/influxdb.png)")
    p.add_argument("--opt-in-label", dest="opt_in_label", help="only report pods with label KEY=VALUE")
    p.add_argument("--user-regex", dest="user_regex", help="regex on pod name; group 1 = user")
    p.add_argument("--pod-labels", dest="pod_label_allowlist",
                   help="comma-separated pod label keys exported on pod_gpu_* series as label_<key>")
    p.add_argument("--user-label", dest="user_label", help="pod label holding the user name")
    p.add_argument("--procfs-root", "--procfs", dest="procfs_root")
    p.add_argument("--cri-socket", "--cri", dest="cri_socket")
    p.add_argument("--no-cri", dest="cri_socket", action="store_const", const="none",
                   help="no CRI runtime lookup (kubelet PodResources / log tree / Docker only)")
    p.add_argument("--docker-socket", "--docker", dest="docker_socket",
                   help="plain-Docker nodes: read container names/labels from the Docker Engine API (opt-in)")
    p.add_argument("--pod-resources-socket", "--pod-resources", dest="pod_resources_socket")
    p.add_argument("--no-pod-resources", dest="pod_resources_socket", action="store_const", const="",
                   help="no kubelet PodResources polling (no idle-allocation rows)")
    p.add_argument("--pod-log-root", "--pod-logs", dest="pod_log_root",
                   help="non-root metadata: the kubelet's log tree (containers/ + pods/), e.g. /var/log")
    p.add_argument("--device-checkpoint", dest="device_checkpoint",
                   help="GPU allocations from the kubelet's device-plugin checkpoint file (root-readable)")
    p.add_argument("--control-plane", dest="control_plane", choices=["native", "off"],
                   help="kubelet PodResources / CRI / Docker metadata pollers: native (C++) or off")
    p.add_argument("--no-processes", dest="processes", action="store_false", default=None)
    p.add_argument("--no-gzip", dest="gzip", action="store_false", default=None)
    p.add_argument("--metrics-include", dest="metrics_include",
                   help="comma-separated globs: serve only these metric families (e.g. 'node_gpu_*,pod_gpu_*')")
    p.add_argument("--metrics-exclude", dest="metrics_exclude",
                   help="comma-separated globs: metric families left out of /metrics (e.g. 'gpu_xcd_*')")
    p.add_argument("--dra-drivers", dest="dra_drivers",
                   help="comma-separated DRA driver names whose claims are GPU allocations ('none' = off)")
    p.add_argument("--ras-every", dest="ras_every", type=int, help="RAS error counters every N ticks")
    p.add_argument("--ras-slices", dest="ras_slices", type=int, help="RAS blocks read in N slices over N ticks")
    p.add_argument("--influx-token", dest="influx_token", help="InfluxDB 2.x / 3.x API token (default $INFLUXDB_TOKEN)")
    p.add_argument("--sample-threads", dest="sample_threads", type=int)
    p.add_argument("--rt-priority", dest="rt_priority", type=int)
    p.add_argument("--http-rt-priority", dest="http_rt_priority", type=int,
                   help="SCHED_FIFO priority of the HTTP loops (0 = normal; needs CAP_SYS_NICE)")
    p.add_argument("--http-threads", dest="http_threads", type=int, help="HTTP loop threads serving /metrics")
    p.add_argument("--tls-cert-file", dest="tls_cert_file", help="serve /metrics over HTTPS: PEM certificate chain")
    p.add_argument("--tls-key-file", dest="tls_key_file", help="... and its PEM private key")
    p.add_argument("--tls-client-ca-file", dest="tls_client_ca_file",
                   help="mutual TLS: scrapers must present a certificate signed by this PEM CA")
    p.add_argument("--http-auth-token-file", dest="http_auth_token_file",
                   help="/metrics needs 'Authorization: Bearer <token>', the token read from this file")
    p.add_argument("--prewarm-ms", dest="prewarm_ms", type=float,
                   help="device workers warm the firmware-table read this long before each tick (0 = off)")
    p.add_argument("--device-timeout", dest="device_timeout_s", type=float,
                   help="seconds before a device call is exported as hung (gpu_up 0)")
    p.add_argument("--enable-probe-kernel", "--probe", dest="enable_probe", action="store_true", default=None)
    p.add_argument("--probe-every", dest="probe_every", type=int, help="K1 probe every N ticks")
    p.add_argument("--enable-pmc", "--pmc", dest="enable_pmc", action="store_true", default=None)
    p.add_argument("--pmc-counters", dest="pmc_counters", help="comma-separated PMC counters (default: the built-in set)")
    p.add_argument("--pmc-mode", dest="pmc_mode", choices=["continuous", "window"])
    p.add_argument("--plugin-dir", dest="plugin_dir", help="directory holding libgpumon_pmc.so / libgpumon_probe.so")
    p.add_argument("--no-fast-path", dest="fast_path", action="store_false", default=None,
                   help="amdsmi: read every value through libamd_smi (disable the sysfs/KFD fast path)")
    p.add_argument("--sysfs-root", "--sysfs", dest="sysfs_root")
    p.add_argument("--roctx", dest="roctx", action="store_true", default=None,
                   help="bracket sampler phases with ROCTx ranges (view with rocprofv3 --marker-trace)")
    p.add_argument("--compat", action="store_true",
                   help="reference behaviour: opt-in label mlgpu=mlgpu and 10 s interval")
    p.add_argument("--log-level", dest="log_level")


def from_args(ns: argparse.Namespace, env: Optional[Dict[str, str]] = None) -> Config:
    cfg = Config()
    if getattr(ns, "config", ""):
        cfg.apply_dict(load_yaml(ns.config))
    cfg.apply_env(env)
    if getattr(ns, "compat", False):
        cfg.opt_in_label = cfg.opt_in_label or "mlgpu=mlgpu"
        cfg.interval = 10.0
    names = {f.name: f for f in dataclasses.fields(cfg)}
    for k, v in vars(ns).items():
        if k in names and v is not None:
            if k == "dra_drivers" and v == "none":
                v = ""
            setattr(cfg, k, _coerce(names[k], v))
    return cfg
