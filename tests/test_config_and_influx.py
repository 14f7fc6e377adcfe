"""Config precedence (defaults < YAML < env < flags, reference env names kept) and the InfluxDB
compat push (reference: one requests.post per line, gpu.py:145,218,252; here one batched POST per
tick over keep-alive, received by a local HTTP sink)."""

import argparse
import http.server
import threading
import time

import pytest

from gpumon.config import Config, add_cli_args, from_args


def _ns(argv, env=None):
    p = argparse.ArgumentParser()
    add_cli_args(p)
    return from_args(p.parse_args(argv), env=env or {})


def test_defaults():
    c = Config()
    assert c.interval == 1.0 and c.listen == "0.0.0.0:9400" and c.backend == "auto"
    assert c.opt_in_label == "" and c.user_prefix == "turing-gpu-notebook-"


def test_reference_env_names():
    c = _ns([], env={"NODE_NAME": "gpu02", "INFLUXDB_URL": "http://influx:8086/write?db=k8s"})
    assert c.resolved_host() == "gpu02"
    assert c.influx_url == "http://influx:8086/write?db=k8s"
    core = c.to_core()
    assert core["host"] == "gpu02" and core["influx_url"].endswith("db=k8s")


def test_host_fallback_is_not_none(monkeypatch):
    """Q1: the reference emitted host=None when NODE_NAME was unset."""
    monkeypatch.delenv("NODE_NAME", raising=False)
    h = Config().resolved_host()
    assert h and h != "None"


def test_yaml_env_flag_precedence(tmp_path):
    y = tmp_path / "c.yaml"
    y.write_text("gpumon:\n  interval: 5\n  listen: 0.0.0.0:9000\n  devices: [0, 2]\n  opt_in_label: a=b\n")
    c = _ns(["--config", str(y)], env={})
    assert (c.interval, c.listen, c.devices, c.opt_in_label) == (5.0, "0.0.0.0:9000", [0, 2], "a=b")
    c = _ns(["--config", str(y)], env={"GPUMON_INTERVAL": "2"})
    assert c.interval == 2.0
    c = _ns(["--config", str(y), "--interval", "0.1"], env={"GPUMON_INTERVAL": "2"})
    assert c.interval == 0.1


def test_compat_flag():
    c = _ns(["--compat"])
    assert c.opt_in_label == "mlgpu=mlgpu" and c.interval == 10.0


def test_unknown_yaml_key_rejected(tmp_path):
    y = tmp_path / "c.yaml"
    y.write_text("bogus: 1\n")
    with pytest.raises(ValueError):
        _ns(["--config", str(y)])


def test_to_core_roundtrip_starts(core):
    c = Config(backend="mock:gpus=3", listen="127.0.0.1:0", interval=0)
    ex = core.Exporter(c.to_core())
    ex.start()
    try:
        assert len(ex.statics()) == 3
    finally:
        ex.stop()


class _Sink(http.server.BaseHTTPRequestHandler):
    bodies = []
    protocol_version = "HTTP/1.1"

    def do_POST(self):  # noqa: N802
        n = int(self.headers.get("Content-Length", 0))
        _Sink.bodies.append((self.path, self.rfile.read(n).decode()))
        self.send_response(204)
        self.send_header("Content-Length", "0")
        self.end_headers()

    def log_message(self, *a):
        pass


def test_influx_batched_push(core):
    _Sink.bodies = []
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _Sink)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    url = f"http://127.0.0.1:{srv.server_address[1]}/write?db=gpu_process"
    ex = core.Exporter({"backend": "mock:gpus=2", "serve_http": False, "interval_s": 0.05,
                        "influx_url": url, "host": "node9", "influx_extended": True})
    ex.start()
    try:
        deadline = time.time() + 5
        while time.time() < deadline and len(_Sink.bodies) < 3:
            time.sleep(0.02)
        st = ex.self_stats()
    finally:
        ex.stop()
        srv.shutdown()
    assert len(_Sink.bodies) >= 3
    path, body = _Sink.bodies[0]
    assert path == "/write?db=gpu_process"
    lines = body.strip().split("\n")
    # one POST per tick carries every line of that tick (reference: one POST per line)
    assert sum(l.startswith("node_gpu,host=node9,gpu_id=") for l in lines) == 2
    assert sum(l.startswith("gpu_ext,") for l in lines) == 2
    assert st["influx_ok"] >= 3 and st["influx_fail"] == 0


def test_influx_unreachable_does_not_block_sampling(core):
    ex = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0.02,
                        "influx_url": "http://127.0.0.1:9/write", "influx_timeout_s": 0.2})
    ex.start()
    try:
        time.sleep(0.5)
        st = ex.self_stats()
    finally:
        ex.stop()
    assert st["ticks"] >= 10  # sampler kept its cadence
    assert st["influx_fail"] + st["influx_dropped"] >= 1
