"""bin/gpumon-exporter as its own process, read through its loopback introspection server.

The image's ENTRYPOINT is the native binary (deploy/Dockerfile), and in a cluster it always
attributes *other* processes: the tenants' (the reference likewise ran as its own container and
listed other containers' GPU processes, /root/reference/Dockerfile:7, gpu.py:174-178). A bench or
test that wants the shipped exporter's numbers runs it the same way: this class writes a config
file with the DaemonSet's keys, starts the binary, and reads the exact tick log, per-scrape service
times, samples, pod rows and self stats from ``debug_listen`` (csrc/core/exporter_debug.cpp).
CPU and memory come from ``/proc/<pid>``: every thread of that process is the exporter's.

Start it before the calling process's first HIP call (``torch.cuda.is_available()`` initialises
HIP): the child is then forked from a process with no GPU state at all.
"""

from __future__ import annotations

import atexit
import http.client
import json
import os
import signal
import socket
import subprocess
import time
from typing import Any, Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BINARY = os.path.join(ROOT, "bin", "gpumon-exporter")
DAEMONSET = os.path.join(ROOT, "deploy", "k8s", "gpumon-daemonset.yaml")


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def daemonset_config(path: str = DAEMONSET) -> Dict[str, Any]:
    """The ``gpumon:`` mapping of the DaemonSet's ConfigMap (the shipped default configuration)."""
    import yaml

    with open(path, "r", encoding="utf-8") as fh:
        for doc in yaml.safe_load_all(fh):
            if isinstance(doc, dict) and doc.get("kind") == "ConfigMap":
                text = next(iter(doc.get("data", {}).values()), "")
                return (yaml.safe_load(text) or {}).get("gpumon", {})
    raise ValueError(f"{path}: no ConfigMap")


def _yaml_value(v: Any) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return repr(v)
    if isinstance(v, (list, tuple)):
        return "[" + ", ".join(_yaml_value(x) for x in v) + "]"
    # a double-quoted scalar the native YAML subset reads (options.cpp: backslash escapes \\ \" \n \t;
    # no \u escapes there, so non-ASCII text stays as UTF-8)
    return json.dumps(str(v), ensure_ascii=False)


def write_config(cfg: Dict[str, Any], path: str) -> None:
    with open(path, "w", encoding="utf-8") as fh:
        fh.write("gpumon:\n")
        for k, v in cfg.items():
            fh.write(f"  {k}: {_yaml_value(v)}\n")


class ChildExporterError(RuntimeError):
    pass


class ChildExporter:
    """One ``bin/gpumon-exporter --config <file>`` child plus a client for its /debug views."""

    def __init__(self, cfg: Dict[str, Any], workdir: str, binary: str = BINARY,
                 env: Optional[Dict[str, str]] = None):
        self.cfg = dict(cfg)
        self.workdir = workdir
        self.binary = binary
        self.env = env
        self.proc: Optional[subprocess.Popen] = None
        self.port = -1
        self.debug_port = -1
        self._conn: Optional[http.client.HTTPConnection] = None
        self.log_path = os.path.join(workdir, "gpumon-exporter.log")

    # ------------------------------------------------------------------ lifecycle
    def start(self, timeout_s: float = 60.0) -> "ChildExporter":
        if not os.access(self.binary, os.X_OK):
            raise ChildExporterError(f"{self.binary} is not built (make core)")
        os.makedirs(self.workdir, exist_ok=True)
        last = ""
        for _ in range(3):  # a port taken between free_port() and the child's bind: new ports
            self.port, self.debug_port = free_port(), free_port()
            cfg = dict(self.cfg, listen=f"127.0.0.1:{self.port}", debug_listen=f"127.0.0.1:{self.debug_port}")
            path = os.path.join(self.workdir, "gpumon-config.yaml")
            write_config(cfg, path)
            env = dict(os.environ if self.env is None else self.env)
            for k in list(env):  # the file is the whole configuration (no GPUMON_* / INFLUXDB_* leaking in)
                if k.startswith("GPUMON_") or k.startswith("INFLUXDB_"):
                    env.pop(k)
            with open(self.log_path, "ab") as log:
                self.proc = subprocess.Popen([self.binary, "--config", path], stdout=log, stderr=subprocess.STDOUT,
                                             env=env, cwd=self.workdir)
            try:
                self._wait_ready(timeout_s)
                # a caller that dies on an exception (bench.py's SystemExit paths) must not leave
                # the exporter running: stop it at interpreter exit too (stop() is idempotent)
                atexit.register(self.stop)
                return self
            except ChildExporterError as e:
                last = str(e)
                self.stop()
                if "in use" not in last:
                    break
        raise ChildExporterError(last)

    def _wait_ready(self, timeout_s: float) -> None:
        t_end = time.monotonic() + timeout_s
        while time.monotonic() < t_end:
            if self.proc.poll() is not None:
                raise ChildExporterError(f"gpumon-exporter exited with {self.proc.returncode}: {self.log_tail()}")
            try:
                st = self.get("/debug/state", timeout=2.0)
                if st.get("seq", 0) >= 1:
                    return
            except (OSError, http.client.HTTPException, ValueError):
                self._conn = None
            time.sleep(0.05)
        raise ChildExporterError(f"gpumon-exporter not ready after {timeout_s:g} s: {self.log_tail()}")

    def log_tail(self, n: int = 2000) -> str:
        try:
            with open(self.log_path, "rb") as fh:
                return fh.read()[-n:].decode(errors="replace").strip()
        except OSError:
            return ""

    def stop(self, timeout_s: float = 15.0) -> Optional[int]:
        if self._conn is not None:
            self._conn.close()
            self._conn = None
        if self.proc is None or self.proc.poll() is not None:
            return None if self.proc is None else self.proc.returncode
        self.proc.send_signal(signal.SIGTERM)
        try:
            return self.proc.wait(timeout_s)
        except subprocess.TimeoutExpired:
            self.proc.kill()
            return self.proc.wait(10)

    @property
    def pid(self) -> int:
        return self.proc.pid if self.proc is not None else -1

    # ------------------------------------------------------------------ /debug client
    def get(self, path: str, timeout: float = 10.0) -> Any:
        for attempt in (0, 1):
            if self._conn is None:
                self._conn = http.client.HTTPConnection("127.0.0.1", self.debug_port, timeout=timeout)
            self._conn.timeout = timeout
            if self._conn.sock is not None:
                self._conn.sock.settimeout(timeout)
            try:
                self._conn.request("GET", path)
                r = self._conn.getresponse()
                body = r.read()
                if r.status != 200:
                    raise ChildExporterError(f"GET {path}: HTTP {r.status}")
                return json.loads(body)
            except (OSError, http.client.HTTPException):
                self._conn.close()
                self._conn = None
                if attempt:
                    raise
        return None

    def state(self) -> dict:
        return self.get("/debug/state")

    @property
    def seq(self) -> int:
        return int(self.get("/debug/state")["seq"])

    def wait_for_seq(self, seq: int, timeout_s: float) -> bool:
        return bool(self.get(f"/debug/wait?seq={int(seq)}&timeout_s={timeout_s:g}", timeout=timeout_s + 10)["ok"])

    def wait_ticks(self, n: int = 1, timeout_s: float = 30.0) -> bool:
        return self.wait_for_seq(self.seq + n, timeout_s)

    def ticks(self, since: int = 0) -> List[dict]:
        return self.get(f"/debug/ticks?since={int(since)}")

    def scrape_count(self) -> int:
        return int(self.get("/debug/state")["scrape_count"])

    def scrape_durations_since(self, n0: int) -> List[float]:
        return list(self.get(f"/debug/scrapes?since={int(n0)}")["durations_s"])

    def statics(self) -> List[dict]:
        return self.get("/debug/state")["statics"]

    def self_stats(self) -> dict:
        return self.get("/debug/state")["self"]

    def samples(self) -> List[dict]:
        return self.get("/debug/samples")

    def pod_rows(self) -> List[dict]:
        return self.get("/debug/rows")

    def procs(self) -> List[dict]:
        """Every GPU context of the last tick, ``row`` false for the hidden ones."""
        return self.get("/debug/procs")

    def metrics(self, timeout: float = 10.0) -> str:
        c = http.client.HTTPConnection("127.0.0.1", self.port, timeout=timeout)
        try:
            c.request("GET", "/metrics")
            r = c.getresponse()
            return r.read().decode()
        finally:
            c.close()

    # ------------------------------------------------------------------ /proc/<pid>
    def threads_cpu(self) -> Dict[str, float]:
        """CPU seconds per thread name (schedstat ns, else clock ticks), summed over same-named threads."""
        return threads_cpu(self.pid)

    def cpu_s(self) -> float:
        return sum(self.threads_cpu().values())

    def rss_bytes(self) -> Optional[int]:
        try:
            with open(f"/proc/{self.pid}/status") as fh:
                for line in fh:
                    if line.startswith("VmRSS:"):
                        return int(line.split()[1]) * 1024
        except OSError:
            pass
        return None


def threads_cpu(pid: int, name_prefix: str = "") -> Dict[str, float]:
    hz = os.sysconf("SC_CLK_TCK")
    out: Dict[str, float] = {}
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for t in tids:
        try:
            with open(f"/proc/{pid}/task/{t}/stat") as fh:
                s = fh.read()
            name = s[s.index("(") + 1:s.rindex(")")]
            if name_prefix and not name.startswith(name_prefix):
                continue
            try:
                with open(f"/proc/{pid}/task/{t}/schedstat") as fh:
                    sec = int(fh.read().split()[0]) * 1e-9
            except (OSError, ValueError, IndexError):
                f = s.rsplit(")", 1)[1].split()
                sec = (int(f[11]) + int(f[12])) / hz
            out[name] = out.get(name, 0.0) + sec
        except (OSError, ValueError):
            continue
    return out
