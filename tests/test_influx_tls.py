"""HTTPS for the InfluxDB compat push, and loud failure for push URLs the exporter cannot use.

Reference: every line goes out with requests.post(INFLUXDB_URL, ...) (/root/reference/gpu.py:20,
145,218,252). requests takes https:// URLs and verifies the server certificate against the system
bundle. InfluxDB 2.x / 3.x Cloud endpoints are TLS-only. Here the push dlopens OpenSSL 3
(csrc/core/tls.cpp) and verifies by default. `influx_ca_file` replaces the bundle and
`influx_tls_insecure` opts out. A URL or TLS setting that cannot work stops both entry points at
startup (exit 2) instead of leaving an exporter whose push never runs.

The TLS sink is Python's `ssl` module. Its certificates come from the `openssl` CLI: a test CA, a
server certificate for localhost / 127.0.0.1 / ::1, an unrelated CA, a certificate for another
name, and a client certificate for mutual TLS.
"""

import http.server
import os
import shutil
import signal
import socket
import ssl
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXPORTER = os.path.join(ROOT, "bin", "gpumon-exporter")

pytestmark = pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl CLI needed for test certificates")


def _openssl(*args, cwd):
    subprocess.run(["openssl", *args], cwd=cwd, check=True, capture_output=True, timeout=60)


def _ca(d, name):
    _openssl("req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes", "-days", "2",
             "-keyout", f"{name}.key", "-out", f"{name}.pem", "-subj", f"/CN={name}", cwd=d)


def _leaf(d, name, ca, san, client=False):
    _openssl("req", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes", "-keyout",
             f"{name}.key", "-out", f"{name}.csr", "-subj", f"/CN={name}", cwd=d)
    with open(os.path.join(d, f"{name}.ext"), "w") as fh:
        fh.write("basicConstraints=CA:FALSE\n")
        if san:
            fh.write(f"subjectAltName={san}\n")
        fh.write(f"extendedKeyUsage={'clientAuth' if client else 'serverAuth'}\n")
    _openssl("x509", "-req", "-in", f"{name}.csr", "-CA", f"{ca}.pem", "-CAkey", f"{ca}.key", "-CAcreateserial",
             "-days", "2", "-out", f"{name}.pem", "-extfile", f"{name}.ext", cwd=d)


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("pki"))
    _ca(d, "ca")
    _ca(d, "otherca")
    _leaf(d, "server", "ca", "DNS:localhost,IP:127.0.0.1,IP:::1")
    _leaf(d, "wrongname", "ca", "DNS:influx.elsewhere.example")
    _leaf(d, "client", "ca", "", client=True)
    return {k: os.path.join(d, f"{k}.pem") for k in ("ca", "otherca", "server", "wrongname", "client")} | {
        "server_key": os.path.join(d, "server.key"), "wrongname_key": os.path.join(d, "wrongname.key"),
        "client_key": os.path.join(d, "client.key")}


class _Sink(http.server.BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def do_POST(self):  # noqa: N802
        n = int(self.headers.get("Content-Length", 0))
        body = self.rfile.read(n).decode()
        self.server.posts.append({"path": self.path, "body": body, "peer": self.client_address,
                                  "host": self.headers.get("Host"), "auth": self.headers.get("Authorization")})
        self.send_response(204)
        self.send_header("Content-Length", "0")
        if self.server.close_every and len(self.server.posts) % self.server.close_every == 0:
            self.send_header("Connection", "close")
            self.close_connection = True
        self.end_headers()

    def log_message(self, *a):
        pass


class _TlsSink(http.server.ThreadingHTTPServer):
    daemon_threads = True

    def __init__(self, cert, key, client_ca=None, family=socket.AF_INET, host="127.0.0.1", close_every=0):
        self.address_family = family
        super().__init__((host, 0), _Sink)
        self.close_every = close_every  # every Nth answer says Connection: close (a load balancer)
        self.posts = []
        self.handshake_errors = []
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.load_cert_chain(cert, key)
        if client_ca:
            ctx.verify_mode = ssl.CERT_REQUIRED
            ctx.load_verify_locations(client_ca)
        self.ctx = ctx
        self.port = self.server_address[1]
        self._th = threading.Thread(target=self.serve_forever, daemon=True)

    def get_request(self):
        # handshake in the request thread, not in accept(): a client that fails verification must
        # not stall the listener
        sock, addr = self.socket.accept()
        return self.ctx.wrap_socket(sock, server_side=True, do_handshake_on_connect=False), addr

    def process_request_thread(self, request, client_address):
        try:
            request.do_handshake()
        except (ssl.SSLError, OSError) as e:
            self.handshake_errors.append(str(e))
            self.shutdown_request(request)
            return
        super().process_request_thread(request, client_address)

    def __enter__(self):
        self._th.start()
        return self

    def __exit__(self, *exc):
        self.shutdown()
        self.server_close()


def _wait(pred, timeout=10.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(0.02)
    return pred()


def test_https_push_delivers_the_exact_tick_lines(core, pki):
    """One tick, one POST over TLS, verified against influx_ca_file. The body is byte-for-byte the
    tick's line protocol (node_gpu / pod_gpu, gpu.py:136-146,206-216)."""
    with _TlsSink(pki["server"], pki["server_key"]) as srv:
        url = f"https://127.0.0.1:{srv.port}/write?db=gpu_process"
        ex = core.Exporter({"backend": "mock:gpus=2", "serve_http": False, "interval_s": 0, "host": "node7",
                            "influx_url": url, "influx_ca_file": pki["ca"]})
        ex.start()  # first tick queued
        try:
            assert _wait(lambda: ex.self_stats()["influx_ok"] >= 1), (ex.self_stats(), srv.handshake_errors)
            want = ex.influx_text()
            st = ex.self_stats()
        finally:
            ex.stop()
    assert len(srv.posts) == 1
    p = srv.posts[0]
    assert p["path"] == "/write?db=gpu_process" and p["host"] == f"127.0.0.1:{srv.port}"
    # byte-for-byte the tick's lines; only the timestamp differs (influx_text() stamps "now", the
    # push carries the tick's sample time, one stamp for the whole batch)
    got_lines, want_lines = p["body"].split("\n"), want.split("\n")
    assert [l.rsplit(" ", 1)[0] for l in got_lines] == [l.rsplit(" ", 1)[0] for l in want_lines]
    stamps = {int(l.rsplit(" ", 1)[1]) for l in got_lines if l}
    assert len(stamps) == 1 and abs(stamps.pop() / 1e9 - time.time()) < 60
    assert sum(l.startswith("node_gpu,host=node7,gpu_id=") for l in p["body"].splitlines()) == 2
    assert st["influx_fail"] == 0 and st["influx_up"] == 1 and st["influx_enabled"]


def test_https_keeps_one_connection_across_pushes(core, pki):
    """Keep-alive over TLS: five requests, one TCP connection (one handshake)."""
    with _TlsSink(pki["server"], pki["server_key"]) as srv:
        st, _, err = core.http_request("POST", f"https://localhost:{srv.port}/write?db=x", "m v=1", "", 5.0,
                                       pki["ca"], False, 5)
    assert st == 204, err
    assert len(srv.posts) == 5
    assert len({p["peer"] for p in srv.posts}) == 1
    assert srv.posts[0]["host"] == f"localhost:{srv.port}"


def test_https_reconnects_after_the_server_closes(core, pki):
    """A load balancer in front of InfluxDB answers some requests with Connection: close: the next
    push opens a new connection and handshakes again, and no push is lost or retried twice."""
    with _TlsSink(pki["server"], pki["server_key"], close_every=2) as srv:
        st, _, err = core.http_request("POST", f"https://localhost:{srv.port}/write?db=x", "m v=1", "", 5.0,
                                       pki["ca"], False, 6)
    assert st == 204, err
    assert len(srv.posts) == 6  # exactly once each
    assert len({p["peer"] for p in srv.posts}) == 3  # 2 requests per connection
    assert not srv.handshake_errors


def test_https_to_an_ipv6_literal(core, pki):
    try:
        srv = _TlsSink(pki["server"], pki["server_key"], family=socket.AF_INET6, host="::1")
    except OSError as e:
        pytest.skip(f"no IPv6 loopback: {e}")
    with srv:
        st, _, err = core.http_request("POST", f"https://[::1]:{srv.port}/write", "m v=1", "", 5.0, pki["ca"])
    assert st == 204, err
    assert srv.posts[0]["host"] == f"[::1]:{srv.port}"


@pytest.mark.parametrize("case,want", [
    ("wrong_ca", "certificate verify failed"),
    ("system_bundle", "certificate verify failed"),
    ("wrong_name", "certificate verify failed: hostname mismatch"),
    ("wrong_ip", "certificate verify failed: IP address mismatch"),
])
def test_https_verification_failures_are_named(core, pki, case, want):
    cert, key = (pki["wrongname"], pki["wrongname_key"]) if case.startswith("wrong_") and case != "wrong_ca" \
        else (pki["server"], pki["server_key"])
    ca = {"wrong_ca": pki["otherca"], "system_bundle": ""}.get(case, pki["ca"])
    host = "localhost" if case == "wrong_name" else "127.0.0.1"
    with _TlsSink(cert, key) as srv:
        st, _, err = core.http_request("POST", f"https://{host}:{srv.port}/write", "m v=1", "", 5.0, ca)
    assert st == -1 and want in err, err
    assert not srv.posts


def test_https_insecure_opt_out_skips_verification(core, pki):
    with _TlsSink(pki["wrongname"], pki["wrongname_key"]) as srv:
        st, _, err = core.http_request("POST", f"https://127.0.0.1:{srv.port}/write", "m v=1", "", 5.0, "", True)
    assert st == 204, err


def test_https_mutual_tls(core, pki):
    """A server that requires a client certificate: the push presents influx_client_cert / _key;
    without them the handshake fails and the push counts an error."""
    with _TlsSink(pki["server"], pki["server_key"], client_ca=pki["ca"]) as srv:
        url = f"https://127.0.0.1:{srv.port}/api/v2/write?org=o&bucket=gpu"
        ok = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0, "influx_url": url,
                            "influx_token": "tok-1", "influx_ca_file": pki["ca"],
                            "influx_client_cert": pki["client"], "influx_client_key": pki["client_key"]})
        ok.start()
        try:
            assert _wait(lambda: ok.self_stats()["influx_ok"] >= 1), srv.handshake_errors
        finally:
            ok.stop()
        assert srv.posts[0]["auth"] == "Token tok-1"
        n = len(srv.posts)
        bad = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0, "influx_url": url,
                             "influx_ca_file": pki["ca"], "influx_timeout_s": 1.0})
        bad.start()
        try:
            assert _wait(lambda: bad.self_stats()["influx_fail"] >= 1)
            st = bad.self_stats()
        finally:
            bad.stop()
        assert len(srv.posts) == n and st["influx_up"] == 0


def test_influx_up_gauge_tracks_the_last_push(core, pki, mock_exporter):
    """gpumon_influx_up: absent without a push URL; 0 while the push fails; 1 once it succeeds; the
    last-success timestamp appears with the first success."""
    plain = mock_exporter()
    assert "gpumon_influx_up" not in plain.metrics_text().replace("# HELP gpumon_influx_up", "").replace(
        "# TYPE gpumon_influx_up", "")
    with _TlsSink(pki["server"], pki["server_key"]) as srv:
        failing = mock_exporter(interval_s=0.05, influx_url=f"https://127.0.0.1:{srv.port}/write",
                                influx_ca_file=pki["otherca"], influx_timeout_s=1.0)
        assert _wait(lambda: failing.self_stats()["influx_fail"] >= 1)
        failing.tick()
        text = failing.metrics_text()
        assert "\ngpumon_influx_up{" in text and 'gpumon_influx_up{host="node-a"} 0' in text, text[-3000:]
        assert "gpumon_influx_last_success_timestamp_seconds{" not in text
        good = mock_exporter(interval_s=0.05, influx_url=f"https://127.0.0.1:{srv.port}/write",
                             influx_ca_file=pki["ca"])
        assert _wait(lambda: good.self_stats()["influx_ok"] >= 1)
        good.tick()
        text = good.metrics_text()
        assert 'gpumon_influx_up{host="node-a"} 1' in text
        ts = [l for l in text.splitlines() if l.startswith("gpumon_influx_last_success_timestamp_seconds{")]
        assert ts and abs(float(ts[0].rsplit(" ", 1)[1]) - time.time()) < 60


@pytest.mark.parametrize("url,want", [
    ("ftp://influx:8086/write", "unsupported scheme 'ftp'"),
    ("influx:8086/write", "no http:// or https:// scheme"),
    ("http://:8086/write", "no host"),
    ("http://influx:99999/write", "port out of range"),
    ("https://influx:80x/write", "bad port '80x'"),
    ("http://fd00::1:8086/write", "an IPv6 host needs brackets"),
    ("http://[fd00::1/write", "unterminated [IPv6] literal"),
])
def test_unusable_push_urls_are_named(core, url, want):
    u = core.parse_url(url)
    assert not u["ok"] and want in u["error"], u
    assert want in core.check_push_config(url)


def test_push_config_checks_tls_files_and_token(core, pki, tmp_path):
    assert core.check_push_config("https://influx:8086/write", ca_file=pki["ca"]) == ""
    assert core.check_push_config("https://influx:8086/write") == ""  # system bundle
    assert "cannot read" in core.check_push_config("https://influx/write", ca_file=str(tmp_path / "none.pem"))
    junk = tmp_path / "junk.pem"
    junk.write_text("not a certificate\n")
    assert "cannot load CA file" in core.check_push_config("https://influx/write", ca_file=str(junk))
    assert "cannot load client key" in core.check_push_config(
        "https://influx/write", client_cert=pki["client"], client_key=pki["server_key"])
    assert "cannot load client certificate" in core.check_push_config(
        "https://influx/write", client_cert=str(junk), client_key=pki["client_key"])
    assert "line break" in core.check_push_config("http://influx/write", token="a\r\nX-Evil: 1")
    assert core.check_push_config("") == ""
    # TLS files for an http:// URL: a warning, not an error (the files are not even opened)
    assert core.check_push_config("http://influx/write", ca_file=str(tmp_path / "none.pem")) == ""


def test_empty_default_trust_store_falls_back_to_the_bundles(core, monkeypatch):
    """SSL_CERT_FILE / SSL_CERT_DIR pointing nowhere (a slim image whose OPENSSLDIR holds no certs)
    leaves libssl's default store empty: the context then loads the distribution bundle itself."""
    if not any(os.access(b, os.R_OK) for b in ("/etc/ssl/certs/ca-certificates.crt", "/etc/pki/tls/certs/ca-bundle.crt",
                                              "/etc/ssl/ca-bundle.pem", "/etc/ssl/cert.pem")):
        pytest.skip("no CA bundle on this host")
    monkeypatch.setenv("SSL_CERT_FILE", "/nonexistent/cert.pem")
    monkeypatch.setenv("SSL_CERT_DIR", "/nonexistent/certs")
    assert core.check_push_config("https://influx:8086/write") == ""


@pytest.mark.parametrize("env,want", [
    ({"GPUMON_LIBSSL": "/nonexistent/libssl.so.3"}, "https needs OpenSSL 3"),
    ({"GPUMON_LIBCRYPTO": "/nonexistent/libcrypto.so.3"}, "https needs OpenSSL 3"),
    ({"GPUMON_LIBSSL": "libz.so.1"}, "libssl / libcrypto lack OPENSSL_init_ssl"),
])
def test_unloadable_openssl_is_named_at_startup(env, want):
    """An https URL on a host without a usable OpenSSL 3 stops the exporter at startup with the
    reason. An override names the only library tried: a wrong path does not quietly load the
    default one."""
    r = subprocess.run([EXPORTER, "--backend", "mock:gpus=1", "--listen", "127.0.0.1:0", "--once"],
                       capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, INFLUXDB_URL="https://influx:8086/write", **env))
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert want in r.stderr, r.stderr[-2000:]


def test_http_push_never_loads_openssl():
    """An http:// deployment runs with no OpenSSL at all: the overrides point nowhere and the
    exporter still starts (libssl is opened only for https)."""
    r = subprocess.run([EXPORTER, "--backend", "mock:gpus=1", "--listen", "127.0.0.1:0", "--once"],
                       capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, INFLUXDB_URL="http://127.0.0.1:9/write", GPUMON_LIBSSL="/nonexistent/libssl.so.3",
                                GPUMON_LIBCRYPTO="/nonexistent/libcrypto.so.3"))
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert "node_gpu_gpu_util" in r.stdout


def test_exporter_start_refuses_an_unusable_push(core):
    ex = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0,
                        "influx_url": "ftp://influx/write"})
    with pytest.raises(RuntimeError, match="unsupported scheme 'ftp'"):
        ex.start()
    ex.stop()


@pytest.mark.parametrize("entry", ["native", "python"])
@pytest.mark.parametrize("env,want", [
    ({"INFLUXDB_URL": "ftp://influx:8086/write"}, "unsupported scheme 'ftp'"),
    ({"INFLUXDB_URL": "https://influx:8086/write", "GPUMON_INFLUX_CA_FILE": "/nonexistent/ca.pem"},
     "cannot read /nonexistent/ca.pem"),
])
def test_both_entry_points_exit_2_on_an_unusable_push(entry, env, want):
    cmd = [EXPORTER] if entry == "native" else [sys.executable, "-m", "gpumon", "serve", "--control-plane", "off"]
    cmd += ["--backend", "mock:gpus=1", "--listen", "127.0.0.1:0", "--interval", "0.2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=60, cwd=ROOT,
                       env=dict(os.environ, PYTHONPATH=ROOT, **env))
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert want in r.stderr, r.stderr[-2000:]


@pytest.mark.slow
def test_native_binary_pushes_over_https(pki):
    """The image's entrypoint end to end: INFLUXDB_URL=https://... from the environment, the CA from
    GPUMON_INFLUX_CA_FILE, one POST per tick, no password in the logs."""
    with _TlsSink(pki["server"], pki["server_key"]) as srv:
        env = dict(os.environ, INFLUXDB_URL=f"https://u:pw-secret@localhost:{srv.port}/write?db=k8s",
                   GPUMON_INFLUX_CA_FILE=pki["ca"], NODE_NAME="gpu-node-3")
        p = subprocess.Popen([EXPORTER, "--backend", "mock:gpus=2", "--interval", "0.1", "--listen", "127.0.0.1:0",
                              "--no-pod-resources", "--no-cri", "--log-level", "debug"],
                             env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        try:
            assert _wait(lambda: len(srv.posts) >= 3, 15), srv.handshake_errors
        finally:
            p.send_signal(signal.SIGTERM)
            _, err = p.communicate(timeout=30)
    assert p.returncode == 0, err[-2000:]
    assert "pw-secret" not in err
    bodies = [x["body"] for x in srv.posts]
    assert all(b.startswith("node_gpu,host=gpu-node-3,gpu_id=0 ") for b in bodies), bodies[0][:200]
    assert srv.posts[0]["auth"].startswith("Basic ")


def test_tls_handshake_with_a_silent_peer_is_bounded(core):
    """A peer that accepts TCP and never answers the ClientHello: the handshake gives up after the
    client's timeout (non-blocking socket, poll() against a per-call deadline) with a named error."""
    import time

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    held = []

    def accept():
        c, _ = srv.accept()
        held.append(c)  # read nothing, send nothing

    t = threading.Thread(target=accept, daemon=True)
    t.start()
    t0 = time.monotonic()
    st, _, err = core.http_request("POST", f"https://127.0.0.1:{port}/write", "m v=1", "", 0.5, "", True)
    dt = time.monotonic() - t0
    t.join(5)
    for c in held:
        c.close()
    srv.close()
    assert st == -1 and "handshake with 127.0.0.1 timed out" in err, err
    assert 0.4 < dt < 2.0, dt


def test_tls_slow_but_steady_server_is_served(core, pki):
    """A verifying TLS sink that takes 0.3 s to answer each POST, client timeout 1 s: pushes succeed
    over the kept connection (the per-call deadline is not a per-connection one)."""
    import time

    class Slow(_Sink):
        def do_POST(self):  # noqa: N802
            time.sleep(0.3)
            super().do_POST()

    srv = _TlsSink(pki["server"], pki["server_key"])
    srv.RequestHandlerClass = Slow
    with srv:
        st, _, err = core.http_request("POST", f"https://127.0.0.1:{srv.port}/write", "m v=1", "", 1.0, pki["ca"],
                                       False, 3)
    assert st == 204, err
    assert len(srv.posts) == 3 and len({p["peer"] for p in srv.posts}) == 1


@pytest.mark.parametrize("trigger", ["period", "sighup"])
def test_push_picks_up_a_rotated_ca_without_a_restart(core, pki, tmp_path, monkeypatch, trigger):
    """The InfluxDB server moves to a certificate from a new CA and the mounted CA file is replaced:
    pushes fail verification until the exporter re-stamps its TLS files (on its period, or at once
    after reload_tls(), the entry points' SIGHUP), then resume without a restart, on a new
    connection."""
    import shutil

    monkeypatch.setenv("GPUMON_TLS_RELOAD_S", "0.3" if trigger == "period" else "3600")
    ca_file = tmp_path / "influx-ca.pem"
    shutil.copy(pki["otherca"], ca_file)  # the CA of the server's *next* certificate is not there yet
    with _TlsSink(pki["server"], pki["server_key"]) as srv:
        ex = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0.1,
                            "influx_url": f"https://localhost:{srv.port}/write?db=k8s", "influx_ca_file": str(ca_file),
                            "influx_timeout_s": 1.0})
        ex.start()
        try:
            assert _wait(lambda: ex.self_stats()["influx_fail"] >= 1), ex.self_stats()
            assert not srv.posts
            tmp = tmp_path / "influx-ca.pem.new"
            shutil.copy(pki["ca"], tmp)
            os.replace(tmp, ca_file)  # the kubelet's rename
            if trigger == "sighup":
                ex.reload_tls()
            assert _wait(lambda: len(srv.posts) >= 1, timeout=20.0), (ex.self_stats(), srv.handshake_errors[-2:])
            assert _wait(lambda: ex.self_stats()["influx_up"] == 1)
        finally:
            ex.stop()
