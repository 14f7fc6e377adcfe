"""/metrics over HTTPS (tls_cert_file / tls_key_file; tls_client_ca_file for mutual TLS).

The reference had no scrape endpoint at all (push only, /root/reference/gpu.py:145). Hardened
clusters scrape node agents over TLS: Prometheus `scheme: https` with a `tlsConfig`, sometimes with a
client certificate. The exporter terminates TLS itself, in the same epoll loops, with the OpenSSL 3
it already dlopens for the Influx push (csrc/core/tls.h TlsServer). Covered here:
- a verified scrape, gzip, keep-alive, HEAD, and a body larger than the socket buffer;
- plain HTTP against the TLS port, an untrusted scraper, a missing or wrong client certificate,
  and a client that never finishes its handshake. Each is counted in
  gpumon_http_tls_handshake_failures_total;
- configuration errors at startup, in both entry points.
"""

import gzip
import http.client
import os
import socket
import ssl
import subprocess
import sys
import time

import pytest

from gpumon.export import promtext
from test_influx_tls import _ca, _leaf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXPORTER = os.path.join(ROOT, "bin", "gpumon-exporter")

pytestmark = pytest.mark.skipif(__import__("shutil").which("openssl") is None, reason="openssl CLI needed")


@pytest.fixture(scope="module")
def pki(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("mpki"))
    _ca(d, "ca")
    _ca(d, "clientca")
    _ca(d, "otherca")
    _leaf(d, "server", "ca", "DNS:localhost,IP:127.0.0.1,IP:::1")
    _leaf(d, "scraper", "clientca", "", client=True)
    _leaf(d, "stranger", "otherca", "", client=True)
    p = lambda n: os.path.join(d, n)  # noqa: E731
    return {"ca": p("ca.pem"), "clientca": p("clientca.pem"), "otherca": p("otherca.pem"), "server": p("server.pem"),
            "server_key": p("server.key"),
            "scraper": p("scraper.pem"), "scraper_key": p("scraper.key"), "stranger": p("stranger.pem"),
            "stranger_key": p("stranger.key")}


def _ctx(pki, cert=None, key=None, ca="ca"):
    c = ssl.create_default_context(cafile=pki[ca])
    if cert:
        c.load_cert_chain(pki[cert], pki[key])
    return c


def _get(port, ctx, path="/metrics", headers=None, method="GET", conn=None):
    c = conn or http.client.HTTPSConnection("localhost", port, context=ctx, timeout=5)
    c.request(method, path, headers=headers or {})
    r = c.getresponse()
    body = r.read()
    return r.status, dict(r.getheaders()), body, c


def _failures(ex):
    return promtext.one(promtext.parse(ex.metrics_text()), "gpumon_http_tls_handshake_failures_total")


def test_verified_https_scrape_gzip_keepalive_and_head(mock_exporter, pki):
    ex = mock_exporter(backend="mock:gpus=8", tls_cert_file=pki["server"], tls_key_file=pki["server_key"])
    ex.tick()
    st, h, body, c = _get(ex.port, _ctx(pki))
    assert st == 200 and h["Content-Type"].startswith("text/plain; version=0.0.4")
    assert int(h["Content-Length"]) == len(body) and body.decode() == ex.metrics_text()
    # keep-alive: the next requests ride the same TLS session
    st, h, gz, c = _get(ex.port, None, headers={"Accept-Encoding": "gzip"}, conn=c)
    assert st == 200 and h.get("Content-Encoding") == "gzip" and gzip.decompress(gz) == body
    st, h, b, c = _get(ex.port, None, method="HEAD", conn=c)
    assert st == 200 and b == b"" and int(h["Content-Length"]) == len(body)
    st, _, b, c = _get(ex.port, None, path="/healthz", conn=c)
    assert st == 200 and b == b"ok\n"
    c.close()
    assert ex.self_stats()["http_tls_failures"] == 0
    ex.tick()
    assert _failures(ex) == 0


def test_response_larger_than_the_socket_buffer(core, pki, monkeypatch):
    """An 8-GPU exposition through a 4 KiB send buffer and a reader that stalls: the response goes
    out record by record, resumed from the loop's offset on each EPOLLOUT (partial-write mode)."""
    monkeypatch.setenv("GPUMON_HTTP_SNDBUF", "4096")
    ex = core.Exporter({"backend": "mock:gpus=8", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_threads": 1, "gzip": False, "tls_cert_file": pki["server"],
                        "tls_key_file": pki["server_key"]})
    ex.start()
    try:
        want = ex.metrics_text().encode()
        assert len(want) > 64 * 1024
        raw = socket.create_connection(("127.0.0.1", ex.port))
        raw.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
        s = _ctx(pki).wrap_socket(raw, server_hostname="localhost")
        s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n")
        time.sleep(0.3)  # let the server fill the small buffers and wait on EPOLLOUT
        data = b""
        while b"\r\n\r\n" not in data or len(data) < data.index(b"\r\n\r\n") + 4 + len(want):
            chunk = s.recv(65536)
            assert chunk, len(data)
            data += chunk
        assert data.split(b"\r\n\r\n", 1)[1] == want
        s.close()
    finally:
        ex.stop()


@pytest.mark.parametrize("case", ["plain_http", "untrusted_scraper", "silent_client"])
def test_failed_handshakes_are_counted_and_closed(core, pki, case, monkeypatch):
    monkeypatch.setenv("GPUMON_HTTP_HEADER_TIMEOUT_S", "0.5")
    ex = core.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_threads": 1, "tls_cert_file": pki["server"], "tls_key_file": pki["server_key"]})
    ex.start()
    try:
        if case == "plain_http":
            s = socket.create_connection(("127.0.0.1", ex.port), timeout=5)
            s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n")
            try:
                got = s.recv(4096)  # a TLS alert or nothing, then the close -- never an HTTP answer
            except ConnectionResetError:  # closed with the request unread: a reset
                got = b""
            assert not got.startswith(b"HTTP/")
            s.close()
        elif case == "untrusted_scraper":
            with pytest.raises(ssl.SSLError):
                _get(ex.port, _ctx(pki, ca="otherca"))
        else:
            s = socket.create_connection(("127.0.0.1", ex.port), timeout=5)
            deadline = time.time() + 5
            s.settimeout(0.2)
            closed = False
            while time.time() < deadline and not closed:
                try:
                    closed = s.recv(1) == b""
                except socket.timeout:
                    pass
                except ConnectionResetError:
                    closed = True
            assert closed, "a client that never sends its ClientHello must not hold a slot"
            s.close()
        deadline = time.time() + 5
        while ex.self_stats()["http_tls_failures"] < 1 and time.time() < deadline:
            time.sleep(0.05)
        assert ex.self_stats()["http_tls_failures"] == 1
        # the server still serves a good scraper afterwards
        assert _get(ex.port, _ctx(pki))[0] == 200
    finally:
        ex.stop()


def test_mutual_tls_requires_a_client_certificate_from_the_ca(core, pki):
    """Mutual TLS: a certificate from another CA fails the handshake; a connection WITHOUT a
    certificate is accepted (the kubelet's HTTPS probes send none: ADVICE r5, every probe failed at
    the handshake and restarted the pod), answers /healthz and /readyz, and gets 403 on /metrics."""
    ex = core.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_threads": 1, "tls_cert_file": pki["server"], "tls_key_file": pki["server_key"],
                        "tls_client_ca_file": pki["clientca"]})
    ex.start()
    try:
        assert _get(ex.port, _ctx(pki, "scraper", "scraper_key"))[0] == 200
        # TLS 1.3: the server's refusal may only surface on the first read, as an alert or a reset
        with pytest.raises((ssl.SSLError, ConnectionResetError, http.client.RemoteDisconnected)):
            _get(ex.port, _ctx(pki, "stranger", "stranger_key"))
        deadline = time.time() + 5
        while ex.self_stats()["http_tls_failures"] < 1 and time.time() < deadline:
            time.sleep(0.05)
        assert ex.self_stats()["http_tls_failures"] == 1
        # no client certificate: the probes' view
        for path, want in (("/healthz", 200), ("/readyz", 200), ("/metrics", 403)):
            assert _get(ex.port, _ctx(pki), path)[0] == want, path
        assert ex.self_stats()["http_tls_failures"] == 1  # the probe handshakes all succeeded
        assert ex.self_stats()["http_tls_client_cert_refused"] == 1
        ex.tick()  # the snapshot that carries the counter
        fam = promtext.parse(_get(ex.port, _ctx(pki, "scraper", "scraper_key"))[2].decode())
        assert promtext.one(fam, "gpumon_http_tls_client_cert_refused_total") == 1
    finally:
        ex.stop()


def test_plain_exporter_has_no_tls_family(mock_exporter):
    ex = mock_exporter()
    ex.tick()
    assert "gpumon_http_tls_handshake_failures_total" not in ex.metrics_text()
    assert ex.self_stats()["http_tls_failures"] == -1


@pytest.mark.parametrize("over,want", [
    ({"tls_cert_file": "CERT"}, "tls_cert_file and tls_key_file go together"),
    ({"tls_client_ca_file": "CA"}, "tls_client_ca_file needs tls_cert_file and tls_key_file"),
    ({"tls_cert_file": "CERT", "tls_key_file": "/nonexistent/key.pem"}, "cannot read /nonexistent/key.pem"),
    ({"tls_cert_file": "CERT", "tls_key_file": "OTHERKEY"}, "does not match the certificate"),
    ({"tls_cert_file": "JUNK", "tls_key_file": "KEY"}, "cannot load certificate"),
])
def test_bad_tls_files_fail_at_startup(core, pki, tmp_path, over, want):
    junk = tmp_path / "junk.pem"
    junk.write_text("not a certificate\n")
    sub = {"CERT": pki["server"], "KEY": pki["server_key"], "CA": pki["clientca"], "OTHERKEY": pki["scraper_key"],
           "JUNK": str(junk)}
    cfg = {k: sub.get(v, v) for k, v in over.items()}
    assert want in core.check_serve_tls(cfg.get("tls_cert_file", ""), cfg.get("tls_key_file", ""),
                                        cfg.get("tls_client_ca_file", ""))
    ex = core.Exporter(dict({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0}, **cfg))
    with pytest.raises(RuntimeError, match=want):
        ex.start()
    ex.stop()


@pytest.mark.parametrize("entry", ["native", "python"])
def test_entry_points_serve_https_and_refuse_bad_files(entry, pki):
    base = [EXPORTER] if entry == "native" else [sys.executable, "-m", "gpumon", "serve", "--control-plane", "off"]
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run(base + ["--backend", "mock:gpus=1", "--listen", "127.0.0.1:0", "--tls-cert-file", pki["server"]],
                       capture_output=True, text=True, timeout=60, cwd=ROOT, env=env)
    assert r.returncode == 2 and "tls_cert_file and tls_key_file go together" in r.stderr, (r.returncode, r.stderr)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = subprocess.Popen(base + ["--backend", "mock:gpus=2", "--interval", "0.2", "--listen", f"127.0.0.1:{port}",
                                 "--tls-cert-file", pki["server"], "--tls-key-file", pki["server_key"]],
                         cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        deadline = time.time() + 30
        while True:
            try:
                st, _, body, c = _get(port, _ctx(pki))
                c.close()
                if st == 200 or time.time() > deadline:
                    break  # 503 until the first tick is published (a loaded host: not yet)
            except (OSError, ssl.SSLError):
                assert time.time() < deadline and p.poll() is None, p.stderr.read().decode()[-2000:] if p.poll() else ""
            time.sleep(0.1)
        assert st == 200 and b"node_gpu_gpu_util{" in body
    finally:
        p.terminate()
        p.wait(10)


def test_fleet_view_reads_https_exporters(mock_exporter, pki):
    """`gpumon top --url https://... --ca-file` over an exporter serving TLS."""
    from gpumon.export import fleet

    ex = mock_exporter(tls_cert_file=pki["server"], tls_key_file=pki["server_key"])
    ex.tick()
    frames, errors = fleet.fetch([f"https://localhost:{ex.port}/metrics"], ca_file=pki["ca"])
    assert not errors and len(fleet.gpu_rows(frames[0])) == 2
    frames, errors = fleet.fetch([f"https://localhost:{ex.port}/metrics"], ca_file=pki["otherca"])
    assert not frames and "certificate verify failed" in next(iter(errors.values()))


def test_host_process_without_sigpipe_handling_survives_resets(pki, tmp_path):
    """The exporter embedded in a process that leaves SIGPIPE at its default (fatal) action: TLS
    scrapers that reset the connection mid-response, and Connection: close scrapers that reset
    before the server's close_notify, must not kill it. OpenSSL writes with write(), which has no
    MSG_NOSIGNAL; the HTTP loops block SIGPIPE (common.h block_sigpipe)."""
    script = tmp_path / "host.py"
    script.write_text(f'''
import os, signal, socket, ssl, struct, sys, time
sys.path.insert(0, {ROOT!r})
signal.signal(signal.SIGPIPE, signal.SIG_DFL)
os.environ["GPUMON_HTTP_SNDBUF"] = "4096"
from gpumon import core
ex = core().Exporter({{"backend": "mock:gpus=8", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                      "http_threads": 2, "gzip": False, "tls_cert_file": {pki["server"]!r},
                      "tls_key_file": {pki["server_key"]!r}}})
ex.start()
ctx = ssl.create_default_context(cafile={pki["ca"]!r})
for i in range(60):
    raw = socket.create_connection(("127.0.0.1", ex.port))
    raw.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
    s = ctx.wrap_socket(raw, server_hostname="localhost")
    close = b"Connection: close\\r\\n" if i % 2 else b""
    s.sendall(b"GET /metrics HTTP/1.1\\r\\nHost: x\\r\\n" + close + b"\\r\\n")
    if i % 3 == 0:
        s.recv(100)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
    s.close()
time.sleep(0.5)
ex.stop()
print("alive")
''')
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "alive" in r.stdout, (r.returncode, r.stderr[-2000:])


def test_rotated_certificate_is_picked_up_without_a_restart(core, pki, tmp_path, monkeypatch):
    """cert-manager renews the Secret, the kubelet swaps the mounted files: within the check period
    (5 s; 0.3 s here via GPUMON_TLS_RELOAD_S) new connections get the new certificate (its expiry
    exported), the reload is counted, and a rotation that does not load keeps the previous
    certificate in use."""
    import shutil

    monkeypatch.setenv("GPUMON_TLS_RELOAD_S", "0.3")

    d = tmp_path
    ca_dir = os.path.dirname(pki["ca"])
    # the renewed certificate: same CA and names, a later expiry
    _openssl = lambda *a: subprocess.run(["openssl", *a], cwd=ca_dir, check=True, capture_output=True, timeout=60)  # noqa: E731
    _openssl("req", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1", "-nodes", "-keyout", str(d / "new.key"),
             "-out", str(d / "new.csr"), "-subj", "/CN=server")
    (d / "new.ext").write_text("basicConstraints=CA:FALSE\nsubjectAltName=DNS:localhost,IP:127.0.0.1\n"
                               "extendedKeyUsage=serverAuth\n")
    _openssl("x509", "-req", "-in", str(d / "new.csr"), "-CA", "ca.pem", "-CAkey", "ca.key", "-CAcreateserial",
             "-days", "9", "-out", str(d / "new.pem"), "-extfile", str(d / "new.ext"))
    live = d / "live"
    live.mkdir()

    def install(cert, key):  # the kubelet's way: write elsewhere, then rename into place
        for src, name in ((cert, "tls.crt"), (key, "tls.key")):
            tmp = live / (name + ".tmp")
            shutil.copy(src, tmp)
            os.replace(tmp, live / name)

    install(pki["server"], pki["server_key"])
    ex = core.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_threads": 2, "tls_cert_file": str(live / "tls.crt"), "tls_key_file": str(live / "tls.key")})
    ex.start()
    ctx = _ctx(pki)

    def served_not_after():
        with socket.create_connection(("127.0.0.1", ex.port), timeout=5) as raw:
            with ctx.wrap_socket(raw, server_hostname="localhost") as s:
                return ssl.cert_time_to_seconds(s.getpeercert()["notAfter"])

    try:
        first = served_not_after()
        assert abs(ex.self_stats()["http_tls_not_after"] - first) <= 1
        install(str(d / "new.pem"), str(d / "new.key"))
        deadline = time.time() + 15
        while ex.self_stats()["http_tls_reloads_ok"] < 1 and time.time() < deadline:
            time.sleep(0.2)
        st = ex.self_stats()
        assert st["http_tls_reloads_ok"] == 1, st
        renewed = served_not_after()
        assert renewed - first > 5 * 86400 and abs(st["http_tls_not_after"] - renewed) <= 1
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpumon_http_tls_cert_not_after_timestamp_seconds") == st["http_tls_not_after"]
        assert promtext.one(fam, "gpumon_http_tls_reloads_total", result="ok") == 1
        # a rotation that does not load (a key from another certificate): counted, the old one stays
        install(pki["server"], str(d / "new.key"))
        deadline = time.time() + 15
        while ex.self_stats()["http_tls_reloads_failed"] < 1 and time.time() < deadline:
            time.sleep(0.2)
        assert ex.self_stats()["http_tls_reloads_failed"] == 1
        assert served_not_after() == renewed
    finally:
        ex.stop()


@pytest.mark.parametrize("entry", ["native", "python"])
def test_sighup_reloads_the_certificate_now(entry, pki, tmp_path):
    """`kill -HUP`: both entry points re-check the TLS files within a second, whatever the
    rotation period (an hour here)."""
    import shutil
    import signal

    live = tmp_path / "live"
    live.mkdir()
    shutil.copy(pki["server"], live / "tls.crt")
    shutil.copy(pki["server_key"], live / "tls.key")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    base = [EXPORTER] if entry == "native" else [sys.executable, "-m", "gpumon", "serve", "--control-plane", "off"]
    p = subprocess.Popen(base + ["--backend", "mock:gpus=1", "--interval", "0.2", "--listen", f"127.0.0.1:{port}",
                                 "--tls-cert-file", str(live / "tls.crt"), "--tls-key-file", str(live / "tls.key")],
                         cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT, GPUMON_TLS_RELOAD_S="3600"),
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    ctx = _ctx(pki)

    def reloads():
        st, _, body, c = _get(port, ctx, path="/metrics?include=gpumon_http_tls_reloads_total")
        c.close()
        if st != 200:  # 503 until the first tick is published (a loaded host: not yet)
            raise OSError(f"HTTP {st}")
        return promtext.one(promtext.parse(body.decode()), "gpumon_http_tls_reloads_total", result="ok")

    try:
        deadline = time.time() + 30
        while True:
            try:
                assert reloads() == 0
                break
            except (OSError, ssl.SSLError):
                assert time.time() < deadline and p.poll() is None
                time.sleep(0.1)
        # a re-issued certificate for the same key (same names, new serial): what a renewal installs
        d = os.path.dirname(pki["ca"])
        subprocess.run(["openssl", "x509", "-req", "-in", os.path.join(d, "server.csr"), "-CA", "ca.pem", "-CAkey",
                        "ca.key", "-CAcreateserial", "-days", "3", "-out", str(tmp_path / "renewed.pem"), "-extfile",
                        os.path.join(d, "server.ext")], cwd=d, check=True, capture_output=True, timeout=60)
        os.replace(tmp_path / "renewed.pem", live / "tls.crt")
        time.sleep(1.5)
        assert reloads() == 0  # the hour-long period has not come round
        p.send_signal(signal.SIGHUP)
        deadline = time.time() + 10
        while reloads() < 1:
            assert time.time() < deadline and p.poll() is None
            time.sleep(0.2)
    finally:
        p.terminate()
        p.wait(10)


def test_garbage_after_the_handshake_closes_the_connection(core, pki):
    """Bytes that are not a TLS record after a completed handshake: the session fails, and the server
    closes the connection. A failed session reads nothing more, so the level-triggered readable
    socket must not be left in the loop's epoll set, where it would fire on every wait."""
    ex = core.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_threads": 1, "tls_cert_file": pki["server"], "tls_key_file": pki["server_key"]})
    ex.start()
    try:
        raw = socket.create_connection(("127.0.0.1", ex.port), timeout=5)
        s = _ctx(pki).wrap_socket(raw, server_hostname="localhost")
        raw2 = socket.socket(fileno=s.detach())  # the TCP socket under the finished handshake
        raw2.sendall(b"\x17\x03\x03\x00\x10" + b"not a real record" * 4)
        # the client keeps its end open: the loop must not spin on the readable socket meanwhile
        cpu0, t0 = time.process_time(), time.monotonic()
        time.sleep(1.0)
        burn = (time.process_time() - cpu0) / (time.monotonic() - t0)
        raw2.settimeout(5)
        try:
            while raw2.recv(4096):
                pass  # an alert, then the close
        except (ConnectionResetError, socket.timeout):
            pass
        raw2.close()
        assert burn < 0.3, burn  # a spinning loop burns a whole CPU
        assert _get(ex.port, _ctx(pki))[0] == 200  # the server is fine
        assert ex.self_stats()["http_connections"] <= 1
    finally:
        ex.stop()


@pytest.mark.parametrize("bodies,cap_at", [((60000, 33000, 0), 90112),  # this tree's cap (86016)
                                            ((50000, 25000, 0), 73728)])  # a 64 KiB cap's
def test_pipelined_input_over_the_buffer_cap_is_all_answered(core, pki, monkeypatch, bodies, cap_at):
    """Pipelined requests with bodies, more than the per-connection input cap (80 KiB + 4 KiB) at
    once. The loop stops reading at the cap; over TLS the session then holds the rest of the record
    it was reading, decrypted bytes that no socket event announces (they left the socket). The
    loop must read on after serving, or the last requests wait for the 10 s header timeout.
    The input piles up while the server is busy writing a large /metrics response to a reader that
    does not read (4 KiB buffers), so it is all there when the server turns to it."""
    monkeypatch.setenv("GPUMON_HTTP_SNDBUF", "4096")
    ex = core.Exporter({"backend": "mock:gpus=8", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_threads": 1, "gzip": False, "tls_cert_file": pki["server"],
                        "tls_key_file": pki["server_key"]})
    ex.start()
    try:
        want = ex.metrics_text().encode()

        def req(n):
            return b"GET /healthz HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n" % n + b"b" * n
        # the cap is crossed inside the last 16 KiB record (the loop reads 8 KiB at a time)
        pipelined = b"".join(req(n) for n in bodies)
        assert cap_at < len(pipelined) <= (cap_at // 16384 + 1) * 16384
        raw = socket.create_connection(("127.0.0.1", ex.port), timeout=5)
        raw.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
        raw.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 1 << 20)
        s = _ctx(pki).wrap_socket(raw, server_hostname="localhost")
        s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n")
        time.sleep(0.3)  # the server now waits on EPOLLOUT
        s.sendall(pipelined)
        time.sleep(0.2)
        t0 = time.monotonic()
        data = b""
        while data.count(b"ok\n") < 3:
            chunk = s.recv(65536)
            assert chunk, data[-200:]
            data += chunk
        assert time.monotonic() - t0 < 3  # not held until the header timeout
        assert data.count(b"HTTP/1.1 200") == 4 and want in data
        s.close()
    finally:
        ex.stop()
