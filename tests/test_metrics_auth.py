"""/metrics behind a bearer token (http_auth_token_file, csrc/core/http_auth.h).

The reference served nothing (gpu.py pushed to InfluxDB); gpumon's endpoint can require
`Authorization: Bearer <token>`, which Prometheus sends from `authorization.credentials_file`
(prometheus-operator: `bearerTokenSecret`). The health endpoints stay open for the kubelet's probes.
The token file is a mounted Secret and rotates without a restart, like the TLS files.
"""

import http.client
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

from gpumon.export import promtext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXPORTER = os.path.join(ROOT, "bin", "gpumon-exporter")


def _get(port, token=None, path="/metrics", auth=None):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    h = {}
    if auth is not None:
        h["Authorization"] = auth
    elif token is not None:
        h["Authorization"] = f"Bearer {token}"
    c.request("GET", path, headers=h)
    r = c.getresponse()
    body = r.read()
    c.close()
    return r.status, dict(r.getheaders()), body


def _wait(pred, timeout=10.0):
    end = time.time() + timeout
    while time.time() < end:
        if pred():
            return True
        time.sleep(0.05)
    return pred()


@pytest.fixture
def token_file(tmp_path):
    p = tmp_path / "token"
    p.write_text("s3cr3t-Token_1\n")
    return p


def test_metrics_needs_the_token_and_health_stays_open(mock_exporter, token_file):
    ex = mock_exporter(http_auth_token_file=str(token_file))
    ex.tick()
    st, h, body = _get(ex.port)
    assert st == 401 and h["WWW-Authenticate"] == 'Bearer realm="gpumon"' and b"node_gpu" not in body
    for auth in ("Bearer wrong", "Bearer s3cr3t-Token_", "Bearer s3cr3t-Token_12", "Basic czNjcjN0", "s3cr3t-Token_1",
                 "Bearer", ""):
        assert _get(ex.port, auth=auth)[0] == 401, auth
    st, _, body = _get(ex.port, "s3cr3t-Token_1")
    assert st == 200 and body.decode() == ex.metrics_text()
    # the scheme is case-insensitive (RFC 7235), extra spaces are tolerated
    assert _get(ex.port, auth="bearer   s3cr3t-Token_1 ")[0] == 200
    # a family filter goes through the same check
    assert _get(ex.port, path="/metrics?include=node_gpu_*")[0] == 401
    assert _get(ex.port, "s3cr3t-Token_1", path="/metrics?include=node_gpu_*")[0] == 200
    for path in ("/healthz", "/livez", "/readyz"):
        assert _get(ex.port, path=path)[0] == 200, path
    assert ex.self_stats()["http_auth_failures"] == 9
    ex.tick()
    fams = promtext.parse(ex.metrics_text())
    for reason in ("missing", "scheme", "token"):  # 3 each: see the requests above
        assert promtext.one(fams, "gpumon_http_auth_failures_total", reason=reason) == 3, reason
    assert promtext.one(fams, "gpumon_http_auth_token_reloads_total", result="ok") == 0


def test_open_exporter_has_no_auth_family(mock_exporter):
    ex = mock_exporter()
    ex.tick()
    assert _get(ex.port)[0] == 200
    assert "gpumon_http_auth" not in ex.metrics_text()
    assert ex.self_stats()["http_auth_failures"] == -1


@pytest.mark.parametrize("content,want", [("", "no token in the file"), ("\n\n", "no token in the file"),
                                          ("two words\n", "not visible ASCII"), ("x" * 5000, "longer than 4096")])
def test_unusable_token_files_fail_at_startup(core, tmp_path, content, want):
    p = tmp_path / "token"
    p.write_text(content)
    assert want in core.check_auth_token_file(str(p))
    assert "cannot read" in core.check_auth_token_file(str(tmp_path / "missing"))
    assert core.check_auth_token_file("") == ""
    ex = core.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_auth_token_file": str(p)})
    with pytest.raises(RuntimeError, match=want):
        ex.start()
    ex.stop()


def test_token_file_format(core, tmp_path):
    p = tmp_path / "t"
    p.write_text("  abc.DEF-123~+/=  \r\n")  # kubectl create secret keeps a trailing newline
    assert core.read_token_file(str(p)) == ("", "abc.DEF-123~+/=", ["abc.DEF-123~+/="])
    p.write_text("first\n\n  second \n")  # one token per line, blank lines skipped
    assert core.read_token_file(str(p)) == ("", "first", ["first", "second"])
    p.write_text("".join(f"t{i}\n" for i in range(17)))
    assert "more than 16 tokens" in core.read_token_file(str(p))[0]
    p.write_text("ok\nnot ok\n")
    assert "not visible ASCII" in core.read_token_file(str(p))[0]


def test_rotation_with_an_overlap_refuses_no_scrape(mock_exporter, tmp_path, monkeypatch):
    """The zero-downtime rotation: the new token is added as a second line, the scraper moves to it,
    the old line is dropped. A scraper on either token is served at every step."""
    monkeypatch.setenv("GPUMON_TLS_RELOAD_S", "0.1")
    p = tmp_path / "token"
    p.write_text("token-a\n")
    ex = mock_exporter(http_auth_token_file=str(p), http_threads=2)
    ex.tick()

    def swap(text, scraper):  # the scraper keeps scraping (a reload happens inside a request)
        tmp = tmp_path / "token.new"
        tmp.write_text(text)
        os.replace(tmp, p)
        n = ex.self_stats()["http_auth_reloads_ok"]
        assert _wait(lambda: _get(ex.port, scraper)[0] == 200 and ex.self_stats()["http_auth_reloads_ok"] > n)

    swap("token-a\ntoken-b\n", "token-a")
    assert _get(ex.port, "token-a")[0] == 200 and _get(ex.port, "token-b")[0] == 200
    swap("token-b\n", "token-b")  # the scraper moved to the new token
    assert _get(ex.port, "token-a")[0] == 401 and _get(ex.port, "token-b")[0] == 200
    assert ex.self_stats()["http_auth_failures"] == 1


@pytest.mark.parametrize("trigger", ["period", "sighup"])
def test_rotated_token_is_picked_up_without_a_restart(core, tmp_path, monkeypatch, trigger):
    monkeypatch.setenv("GPUMON_TLS_RELOAD_S", "0.2" if trigger == "period" else "3600")
    p = tmp_path / "token"
    p.write_text("old-token\n")
    ex = core.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_threads": 2, "http_auth_token_file": str(p)})
    ex.start()
    try:
        assert _get(ex.port, "old-token")[0] == 200
        # the kubelet's atomic swap of a Secret volume: a new file renamed over the old one
        tmp = tmp_path / "token.new"
        tmp.write_text("new-token\n")
        os.replace(tmp, p)
        if trigger == "sighup":
            time.sleep(0.3)
            assert _get(ex.port, "old-token")[0] == 200  # no period check for an hour
            ex.reload_tls()
        assert _wait(lambda: _get(ex.port, "new-token")[0] == 200)
        assert _get(ex.port, "old-token")[0] == 401
        # a rotation to an unusable file keeps the token in force
        tmp.write_text("\n")
        os.replace(tmp, p)
        if trigger == "sighup":
            ex.reload_tls()
        assert _wait(lambda: (_get(ex.port, "new-token"), ex.self_stats()["http_auth_reloads_failed"])[1] == 1)
        assert _get(ex.port, "new-token")[0] == 200
        assert ex.self_stats()["http_auth_reloads_ok"] == 1
    finally:
        ex.stop()


def test_token_over_https(core, tmp_path):
    """The token next to TLS (overlays/tls): the header travels encrypted."""
    import ssl

    if __import__("shutil").which("openssl") is None:
        pytest.skip("openssl CLI needed")
    from test_influx_tls import _ca, _leaf

    d = str(tmp_path)
    _ca(d, "ca")
    _leaf(d, "server", "ca", "DNS:localhost,IP:127.0.0.1")
    (tmp_path / "token").write_text("tls-token\n")
    ex = core.Exporter({"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "tls_cert_file": f"{d}/server.pem", "tls_key_file": f"{d}/server.key",
                        "http_auth_token_file": str(tmp_path / "token")})
    ex.start()
    try:
        ctx = ssl.create_default_context(cafile=f"{d}/ca.pem")
        for hdr, want in (({}, 401), ({"Authorization": "Bearer tls-token"}, 200)):
            c = http.client.HTTPSConnection("localhost", ex.port, context=ctx, timeout=5)
            c.request("GET", "/metrics", headers=hdr)
            assert c.getresponse().status == want
            c.close()
    finally:
        ex.stop()


def test_fleet_view_sends_the_token(mock_exporter, token_file):
    from gpumon.export import fleet

    ex = mock_exporter(http_auth_token_file=str(token_file))
    ex.tick()
    url = f"http://127.0.0.1:{ex.port}/metrics"
    frames, errors = fleet.fetch([url])
    assert not frames and errors[url] == "HTTP 401"
    frames, errors = fleet.fetch([url], token="s3cr3t-Token_1")
    assert not errors and len(fleet.gpu_rows(frames[0])) == 2
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "gpumon", "top", "--url", f"127.0.0.1:{ex.port}", "--iterations", "1",
                        "--token-file", str(token_file)], capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 0 and "401" not in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("entry", ["native", "python"])
def test_entry_points_require_the_token_and_refuse_bad_files(entry, token_file, tmp_path):
    base = [EXPORTER] if entry == "native" else [sys.executable, "-m", "gpumon", "serve", "--control-plane", "off"]
    env = dict(os.environ, PYTHONPATH=ROOT)
    empty = tmp_path / "empty"
    empty.write_text("")
    r = subprocess.run(base + ["--backend", "mock:gpus=1", "--listen", "127.0.0.1:0", "--http-auth-token-file", str(empty)],
                       capture_output=True, text=True, timeout=60, cwd=ROOT, env=env)
    assert r.returncode == 2 and "http_auth_token_file" in r.stderr and "no token" in r.stderr, (r.returncode, r.stderr)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # the env spelling, as the DaemonSet sets it
    p = subprocess.Popen(base + ["--backend", "mock:gpus=1", "--interval", "0.2", "--listen", f"127.0.0.1:{port}"],
                         cwd=ROOT, env=dict(env, GPUMON_HTTP_AUTH_TOKEN_FILE=str(token_file)),
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        def up():
            try:
                return _get(port, path="/healthz")[0] == 200
            except OSError:
                assert p.poll() is None, p.stderr.read().decode()[-2000:]
                return False
        assert _wait(up, 30)
        assert _get(port)[0] == 401
        assert _get(port, "s3cr3t-Token_1")[0] == 200
        # SIGHUP re-reads the token file at once
        tmp = tmp_path / "t.new"
        tmp.write_text("rotated\n")
        os.replace(tmp, token_file)
        p.send_signal(signal.SIGHUP)
        assert _wait(lambda: _get(port, "rotated")[0] == 200)
    finally:
        p.terminate()
        p.wait(10)


def test_doctor_checks_the_token_file(tmp_path):
    from gpumon.config import Config
    from gpumon.doctor import FAIL, OK, WARN, auth_token_check

    p = tmp_path / "token"
    p.write_text("0123456789abcdef0123\n")
    p.chmod(0o644)
    st, detail = auth_token_check(Config(http_auth_token_file=str(p)))
    assert st == WARN and "readable by every user" in detail
    p.chmod(0o600)
    assert auth_token_check(Config(http_auth_token_file=str(p)))[0] == OK
    p.write_text("0123456789abcdef0123\nabcdef0123456789abcd\n")
    st, detail = auth_token_check(Config(http_auth_token_file=str(p)))
    assert st == OK and "2 tokens accepted" in detail
    p.write_text("short\n")
    assert auth_token_check(Config(http_auth_token_file=str(p)))[0] == WARN
    p.write_text("\n")
    st, detail = auth_token_check(Config(http_auth_token_file=str(p)))
    assert st == FAIL and "no token" in detail
