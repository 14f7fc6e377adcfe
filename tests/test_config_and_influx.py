"""Config precedence (defaults < YAML < env < flags, reference env names kept) and the InfluxDB
compat push (reference: one requests.post per line, gpu.py:145,218,252; here one batched POST per
tick over keep-alive, received by a local HTTP sink)."""

import argparse
import base64
import os
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
    assert c.interval == 1.0 and c.listen == ":9400" and c.backend == "auto"
    assert c.opt_in_label == "" and c.user_prefix == "turing-gpu-notebook-"


def test_reference_env_names():
    c = _ns([], env={"NODE_NAME": "gpu02", "INFLUXDB_URL": "http://influx:8086/write?db=k8s"})
    assert c.resolved_host() == "gpu02"
    assert c.influx_url == "http://influx:8086/write?db=k8s"
    fin = c.finalized()
    assert fin.host == "gpu02" and c.to_dict()["influx_url"].endswith("db=k8s")


def test_host_fallback_is_not_none(monkeypatch):
    """Q1: the reference emitted host=None when NODE_NAME was unset. One rule, decided in C++
    (csrc/core/options.cpp options_finalize): NODE_NAME, then the host name, then "no_name"."""
    import socket

    monkeypatch.delenv("NODE_NAME", raising=False)
    h = Config().resolved_host()
    assert h and h != "None" and h == (socket.gethostname() or "no_name")


def test_yaml_env_flag_precedence(tmp_path):
    y = tmp_path / "c.yaml"
    y.write_text("gpumon:\n  interval: 5\n  listen: 0.0.0.0:9000\n  devices: [0, 2]\n  opt_in_label: a=b\n")
    c = _ns(["--config", str(y)], env={})
    assert (c.interval, c.listen, c.devices, c.opt_in_label) == (5.0, "0.0.0.0:9000", ["0", "2"], "a=b")
    c = _ns(["--config", str(y)], env={"GPUMON_INTERVAL": "2"})
    assert c.interval == 2.0
    c = _ns(["--config", str(y), "--interval", "0.1"], env={"GPUMON_INTERVAL": "2"})
    assert c.interval == 0.1


def test_compat_flag():
    c = _ns(["--compat"])
    assert c.opt_in_label == "mlgpu=mlgpu" and c.interval == 10.0


def test_unknown_yaml_key_warned_and_ignored(tmp_path, caplog):
    """A file key the exporter does not know is named and ignored -- by both entry points, since
    both parse with csrc/core/options.cpp; a key given from code is an error."""
    y = tmp_path / "c.yaml"
    y.write_text("bogus: 1\ninterval: 3\n")
    with caplog.at_level("WARNING", logger="gpumon"):
        c = _ns(["--config", str(y)])
    assert c.interval == 3 and "'bogus'" in caplog.text
    with pytest.raises(ValueError, match="unknown config key"):
        Config(bogus=1)


def test_finalized_options_start_an_exporter(core):
    c = Config(backend="mock:gpus=3", listen="127.0.0.1:0", interval=0)
    ex = core.Exporter(c.finalized())
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
        # the sink has a body before the client has read its 204 and counted the push
        while time.time() < deadline and (len(_Sink.bodies) < 3 or ex.self_stats()["influx_ok"] < 3):
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


class _GzipSink(_Sink):
    seen = []

    def do_POST(self):  # noqa: N802
        import gzip as _gz

        n = int(self.headers.get("Content-Length", 0))
        raw = self.rfile.read(n)
        enc = self.headers.get("Content-Encoding", "")
        _GzipSink.seen.append((enc, len(raw), (_gz.decompress(raw) if enc == "gzip" else raw).decode()))
        self.send_response(204)
        self.send_header("Content-Length", "0")
        self.end_headers()


def test_influx_gzip_push(core):
    """influx_gzip: each batch goes out with Content-Encoding: gzip (InfluxDB 1.x / 2.x / 3.x decode
    it), several times smaller, and decodes to exactly the plain push's lines."""
    _GzipSink.seen = []
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _GzipSink)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    ex = core.Exporter({"backend": "mock:gpus=8", "serve_http": False, "interval_s": 0, "host": "node9",
                        "influx_url": f"http://127.0.0.1:{srv.server_address[1]}/write?db=k8s", "influx_gzip": True,
                        "influx_extended": True})
    ex.start()
    try:
        deadline = time.time() + 5
        while time.time() < deadline and ex.self_stats()["influx_ok"] < 1:
            time.sleep(0.02)
        want = ex.influx_text()
    finally:
        ex.stop()
        srv.shutdown()
    enc, nbytes, text = _GzipSink.seen[0]
    assert enc == "gzip" and nbytes * 3 < len(text.encode()), (nbytes, len(text))
    strip = lambda t: [l.rsplit(" ", 1)[0] for l in t.strip().split("\n")]  # noqa: E731 (stamps differ)
    assert strip(text) == strip(want)


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


def test_url_parsing_auth_and_v6(core):
    u = core.parse_url("http://influx:8086/write?db=k8s")
    assert (u["ok"], u["host"], u["port"], u["path"], u["auth_header"]) == (True, "influx", 8086, "/write?db=k8s", "")
    u = core.parse_url("http://gpumon:p%40ss:w@influx.monitoring:8086/write?db=k8s")
    assert u["host"] == "influx.monitoring" and u["path"] == "/write?db=k8s"
    assert u["auth_header"] == "Authorization: Basic " + base64.b64encode(b"gpumon:p@ss:w").decode() + "\r\n"
    u = core.parse_url("http://[fd00::1]:8086/api/v2/write?org=o&bucket=b")
    assert (u["ok"], u["host"], u["port"], u["path"]) == (True, "fd00::1", 8086, "/api/v2/write?org=o&bucket=b")
    assert core.parse_url("http://influx?db=x")["path"] == "/?db=x" and core.parse_url("http://influx")["port"] == 80
    for bad in ("ftp://influx:8086/write", "http://:8086/", "http://influx:99999/", "http://influx:80x/",
                "http://[fd00::1/", "http://[fd00::1]x/"):
        assert not core.parse_url(bad)["ok"], bad
    u = core.parse_url("https://influx.example/api/v2/write?org=o")  # TLS: tests/test_influx_tls.py
    assert (u["ok"], u["tls"], u["port"]) == (True, True, 443)
    for b in ("", "f", "fo", "foo", "foob", "fooba", "u:\u00e9\u00fc"):  # padding cases, non-ASCII
        h = core.parse_url(f"http://{b}@h/")["auth_header"]
        assert h == "Authorization: Basic " + base64.b64encode(b.encode()).decode() + "\r\n", b
    assert core.redact_url("http://u:secret@h:1/write?db=x") == "http://u:***@h:1/write?db=x"
    assert core.redact_url("http://u@h/write") == "http://u@h/write"
    assert core.redact_url("http://h/write?u=a@b") == "http://h/write?u=a@b"


def test_python_redact_matches_native(core):
    from gpumon.config import redact_url

    for u in ("http://u:secret@h:1/write?db=x", "http://u@h/write", "http://h/write?u=a@b", "", "h:1",
              "http://u:p@ss@h/write", "http://u:pw@h?db=x", "u:pw@h", "http://u:pw@[fd00::1]:8086/write",
              "http://h:8086/write?db=x", "http://a:b@h/x/y@z"):
        assert redact_url(u) == core.redact_url(u), u


def test_serve_never_logs_the_influx_password(tmp_path):
    """`gpumon serve` (the image's ENTRYPOINT) logged INFLUXDB_URL in full at INFO, so
    1.x credentials in the URL reached the pod logs. Both the Python startup line and the native
    exporter's logs must show the password masked."""
    import signal
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, INFLUXDB_URL="http://gpumon:s3cr3tPW@127.0.0.1:1/write?db=k8s", PYTHONPATH=root)
    p = subprocess.Popen([sys.executable, "-m", "gpumon", "serve", "--backend", "mock:gpus=1", "--listen",
                          "127.0.0.1:0", "--interval", "0.2", "--control-plane", "off", "--log-level", "debug"],
                         cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    time.sleep(3.0)
    p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=30)
    text = out + err
    assert "serving" in text, text[-2000:]
    assert "s3cr3tPW" not in text, text[-2000:]
    assert "gpumon:***@127.0.0.1" in text, text[-2000:]


class _AuthSink(_Sink):
    auth = []

    def do_POST(self):  # noqa: N802
        _AuthSink.auth.append(self.headers.get("Authorization"))
        super().do_POST()


@pytest.mark.parametrize("mode", ["basic", "token"])
def test_influx_push_authenticates(core, mode):
    """InfluxDB with auth on: 1.x credentials from the URL as Basic auth, 2.x/3.x API token from
    influx_token (env INFLUXDB_TOKEN). The reference posted without credentials (gpu.py:145)."""
    _AuthSink.auth, _Sink.bodies = [], []
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _AuthSink)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    cfg = {"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0.05, "host": "n"}
    if mode == "basic":
        cfg["influx_url"] = f"http://gpumon:s3cret@127.0.0.1:{port}/write?db=k8s"
        want = "Basic " + base64.b64encode(b"gpumon:s3cret").decode()
    else:
        cfg.update(influx_url=f"http://127.0.0.1:{port}/api/v2/write?org=o&bucket=gpu", influx_token="tok-123")
        want = "Token tok-123"
    ex = core.Exporter(cfg)
    ex.start()
    try:
        deadline = time.time() + 5
        while time.time() < deadline and len(_AuthSink.auth) < 2:
            time.sleep(0.02)
    finally:
        ex.stop()
        srv.shutdown()
    assert _AuthSink.auth[:2] == [want, want]


def test_influx_credentials_never_printed(tmp_path):
    import json
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, INFLUXDB_URL="http://u:pw123@influx:8086/write?db=k8s", INFLUXDB_TOKEN="tok-456")
    r = subprocess.run([os.path.join(root, "bin/gpumon-exporter"), "--print-config"], capture_output=True,
                       text=True, timeout=30, env=env, check=True)
    assert "pw123" not in r.stdout and "tok-456" not in r.stdout
    d = json.loads(r.stdout)
    assert d["influx_url"] == "http://u:***@influx:8086/write?db=k8s" and d["influx_token"] == "***"
    c = Config().apply_env({"INFLUXDB_TOKEN": "tok-456"})
    assert c.influx_token == "tok-456" and c.to_dict(redact=True)["influx_token"] == "***"


def test_influx_token_with_a_line_break_is_refused_at_start(core):
    """A token is copied into a request header: CR/LF in it would inject headers. The exporter
    refuses to start with it (a configuration error), rather than running without a push."""
    ex = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0.02,
                        "influx_url": "http://127.0.0.1:9/write", "influx_token": "tok\r\nX-Evil: 1"})
    with pytest.raises(RuntimeError, match="influx_token contains a line break"):
        ex.start()
    ex.stop()


def test_devices_accept_hip_ids_and_bdfs_and_refuse_the_rest():
    """`devices` takes hip ids and PCI BDFs (loaders name GPUs by BDF); the core
    gets them normalised, and a token that is neither is a configuration error, as in the binary."""
    from gpumon.config import Config

    assert Config(devices=[0, "75:00.0", "0000:E5:00.0"]).devices == ["0", "0000:75:00.0", "0000:e5:00.0"]
    assert Config().apply_dict({"devices": "1, 0000:25:00.0"}).devices == ["1", "0000:25:00.0"]
    with pytest.raises(ValueError, match="neither a hip id nor a PCI BDF"):
        Config(devices=["gpu3"])


class _FlakySink(_Sink):
    """Answers the first `fail` POSTs with `code`, then 204."""
    fail, code, seen = 0, 503, 0

    def do_POST(self):  # noqa: N802
        n = int(self.headers.get("Content-Length", 0))
        body = self.rfile.read(n).decode()
        _FlakySink.seen += 1
        if _FlakySink.seen <= _FlakySink.fail:
            self.send_response(_FlakySink.code)
            self.send_header("Content-Length", "0")
            self.end_headers()
            return
        _Sink.bodies.append((self.path, body))
        self.send_response(204)
        self.send_header("Content-Length", "0")
        self.end_headers()


@pytest.mark.parametrize("code,kept", [(503, True), (429, True), (400, False)])
def test_influx_transient_failures_are_retried_in_order(core, code, kept):
    """An InfluxDB that answers 503 / 429 for a while (a restart, rate limiting) loses no batch:
    the failed batch goes back to the head of the queue and the push backs off. A 400 is not
    transient: that batch is dropped, the next ones go through."""
    _Sink.bodies = []
    _FlakySink.fail, _FlakySink.code, _FlakySink.seen = 2, code, 0
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), _FlakySink)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    url = f"http://127.0.0.1:{srv.server_address[1]}/write?db=gpu_process"
    ex = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0, "influx_url": url,
                        "host": "n1"})
    ex.start()  # tick 1 queued
    try:
        for _ in range(4):
            ex.tick()  # ticks 2-5
        deadline = time.time() + 10
        want = 5 if kept else 3
        while time.time() < deadline and len(_Sink.bodies) < want:
            time.sleep(0.05)
        st = ex.self_stats()
    finally:
        ex.stop()
        srv.shutdown()
    stamps = [int(b.strip().split("\n")[0].rsplit(" ", 1)[1]) for _, b in _Sink.bodies]
    assert len(stamps) == (5 if kept else 3), stamps
    assert stamps == sorted(stamps)  # delivered in tick order
    assert st["influx_fail"] == 2
