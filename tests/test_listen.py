"""/metrics listen addresses: IPv4, IPv6, dual-stack, and no silent port sharing.

The reference ships a DaemonSet (/root/reference/gpu_monitor.yaml:21-37) that must be scrapeable
on any cluster network, IPv6 single-stack clusters included. The listener (csrc/core/http_server.h)
takes "host:port", "[v6]:port" or ":port". The default ":9400" is one [::] socket with
IPV6_V6ONLY=0, which takes IPv4 scrapes as ::ffff:a.b.c.d and IPv6 scrapes. It falls back to
0.0.0.0 on a kernel without IPv6.

All event loops share one listening socket (EPOLLEXCLUSIVE) and nothing sets SO_REUSEPORT. So a
second exporter on the same port fails with EADDRINUSE. It does not silently take a share of the
scrapes (a `gpumon-exporter` next to `gpumon serve`, or overlapping hostNetwork pods in a rollout).
"""

import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXPORTER = os.path.join(ROOT, "bin", "gpumon-exporter")


def _has_v6_loopback():
    try:
        s = socket.socket(socket.AF_INET6, socket.SOCK_STREAM)
        s.bind(("::1", 0))
        s.close()
        return True
    except OSError:
        return False


needs_v6 = pytest.mark.skipif(not _has_v6_loopback(), reason="no IPv6 loopback in this network namespace")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scrape(host, port, path="/metrics"):
    h = f"[{host}]" if ":" in host else host
    with urllib.request.urlopen(f"http://{h}:{port}{path}", timeout=5) as r:
        return r.status, r.read()


def _refused(host, port):
    fam = socket.AF_INET6 if ":" in host else socket.AF_INET
    s = socket.socket(fam, socket.SOCK_STREAM)
    s.settimeout(2)
    try:
        s.connect((host, port))
        return False
    except OSError:
        return True
    finally:
        s.close()


CASES = [
    # listen, host, port  (ok) | listen, error fragment (refused)
    ("127.0.0.1:9400", "127.0.0.1", 9400),
    ("0.0.0.0:9400", "0.0.0.0", 9400),
    (":9400", "", 9400),
    ("*:9400", "", 9400),
    ("9400", "", 9400),
    ("[::]:9400", "::", 9400),
    ("[::1]:0", "::1", 0),
    ("[fd00::12]:9100", "fd00::12", 9100),
    ("localhost:8080", "localhost", 8080),
    (" :9400 ", "", 9400),
]
BAD = [
    ("", "empty listen address"),
    ("::1:9400", "needs brackets"),
    ("[::1]", "expected [v6]:port"),
    ("[::1]9400", "expected [v6]:port"),
    ("[nope]:9400", "is not an IPv6 address"),
    ("host", "expected host:port"),
    ("host:", "bad port ''"),
    ("host:99999", "bad port '99999'"),
    ("host:12a", "bad port '12a'"),
]


@pytest.mark.parametrize("listen,host,port", CASES)
def test_parse_listen_native_and_python_agree(core, listen, host, port):
    from gpumon.config import Config, parse_listen

    assert tuple(core.parse_listen(listen)) == (True, host, port, "")
    assert parse_listen(listen) == (host, port)
    c = Config(listen=listen)
    assert (c.listen_addr, c.port) == (host, port)
    assert c.finalized().listen_addr == host


@pytest.mark.parametrize("listen,want", BAD)
def test_parse_listen_refusals_agree(core, listen, want):
    from gpumon.config import ConfigError, parse_listen

    ok, _, _, err = core.parse_listen(listen)
    assert not ok and want in err, err
    with pytest.raises(ConfigError, match=want.replace("[", r"\[").replace("]", r"\]")):
        parse_listen(listen)


def test_default_listen_is_dual_stack_every_address():
    from gpumon.config import Config

    assert Config().listen == ":9400" and Config().listen_addr == ""


@needs_v6
@pytest.mark.parametrize("addr", ["", "::"])
def test_one_dual_stack_listener_serves_ipv4_and_ipv6(mock_exporter, addr):
    ex = mock_exporter(listen_addr=addr, port=0)
    ex.tick()
    assert ex.listen_desc == f"[::]:{ex.port} (dual-stack)"
    st4, b4 = _scrape("127.0.0.1", ex.port)
    st6, b6 = _scrape("::1", ex.port)
    assert st4 == st6 == 200 and b"node_gpu_gpu_util{" in b4 and b"node_gpu_gpu_util{" in b6


@needs_v6
def test_v6_loopback_listener_is_v6_only(mock_exporter):
    ex = mock_exporter(listen_addr="::1", port=0)
    assert ex.listen_desc == f"[::1]:{ex.port}"
    assert _scrape("::1", ex.port)[0] == 200
    assert _refused("127.0.0.1", ex.port)


@needs_v6
def test_ipv4_wildcard_stays_ipv4_only(mock_exporter):
    ex = mock_exporter(listen_addr="0.0.0.0", port=0)
    assert ex.listen_desc == f"0.0.0.0:{ex.port}"
    assert _scrape("127.0.0.1", ex.port)[0] == 200
    assert _refused("::1", ex.port)


def test_host_name_listener_binds_its_first_address(mock_exporter):
    """A host name (a node's own name in `listen`) is resolved once at startup and the listener binds
    its first address; the log names that address, not the name."""
    ex = mock_exporter(listen_addr="localhost", port=0)
    desc = ex.listen_desc
    assert desc in (f"127.0.0.1:{ex.port}", f"[::1]:{ex.port}"), desc
    host = "::1" if desc.startswith("[") else "127.0.0.1"
    assert _scrape(host, ex.port)[0] == 200


def test_unresolvable_listen_host_is_named(core):
    ex = core.Exporter({"backend": "mock:gpus=1", "interval_s": 0, "listen_addr": "no-such-host.invalid", "port": 0})
    with pytest.raises(RuntimeError, match="no-such-host.invalid"):
        ex.start()
    ex.stop()


def _spawn(entry, listen, env_extra=None):
    if entry == "native":
        cmd = [EXPORTER, "--no-pod-resources", "--no-cri"]
    else:
        cmd = [sys.executable, "-m", "gpumon", "serve", "--control-plane", "off"]
    cmd += ["--backend", "mock:gpus=1", "--interval", "0.2", "--listen", listen, "--log-level", "info"]
    return subprocess.Popen(cmd, cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT, **(env_extra or {})),
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def _wait_up(host, port, p, timeout=30):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if p.poll() is not None:
            raise AssertionError(p.communicate()[1][-2000:])
        try:
            if _scrape(host, port, "/healthz")[0] == 200:
                return
        except OSError:
            time.sleep(0.1)
    raise AssertionError("exporter did not come up")


def _stop(p):
    p.send_signal(signal.SIGTERM)
    try:
        return p.communicate(timeout=30)
    except subprocess.TimeoutExpired:
        p.kill()
        return p.communicate()


@needs_v6
@pytest.mark.parametrize("entry", ["native", "python"])
@pytest.mark.parametrize("form", ["[::]:{p}", ":{p}"])
def test_entry_points_serve_both_families(entry, form):
    port = _free_port()
    p = _spawn(entry, form.format(p=port))
    try:
        _wait_up("127.0.0.1", port, p)
        assert _scrape("::1", port)[0] == 200
    finally:
        _, err = _stop(p)
    if entry == "native":
        assert f"serving http://[::]:{port} (dual-stack)/metrics" in err, err[-2000:]


@pytest.mark.parametrize("first,second", [("native", "native"), ("python", "python"), ("python", "native"),
                                          ("native", "python")])
def test_a_second_exporter_on_the_port_fails_loudly(first, second):
    """Two exporters on one fixed port: the second exits non-zero naming EADDRINUSE, and every
    scrape still reaches the first (SO_REUSEPORT would have split them between the two)."""
    port = _free_port()
    a = _spawn(first, f"127.0.0.1:{port}", {"NODE_NAME": "first"})
    try:
        _wait_up("127.0.0.1", port, a)
        b = _spawn(second, f"127.0.0.1:{port}", {"NODE_NAME": "second"})
        try:
            rc = b.wait(timeout=60)
        except subprocess.TimeoutExpired:
            _stop(b)
            raise AssertionError("the second exporter kept running on a taken port")
        err = b.stderr.read()
        assert rc != 0 and "Address already in use" in err, (rc, err[-2000:])
        for _ in range(20):
            assert b'host="first"' in _scrape("127.0.0.1", port)[1]
    finally:
        _stop(a)


def test_dual_stack_default_conflicts_with_an_ipv4_listener():
    """The default ":port" ([::], V6ONLY=0) also claims the IPv4 port: an IPv4 listener already on
    it makes the exporter fail instead of serving only IPv6 next to it."""
    s = socket.socket()
    s.bind(("0.0.0.0", 0))
    s.listen(1)
    port = s.getsockname()[1]
    try:
        p = _spawn("native", f":{port}")
        rc = p.wait(timeout=60)
        assert rc != 0 and "Address already in use" in p.stderr.read()
    finally:
        s.close()


def test_scrape_latency_unchanged_with_the_shared_listener(mock_exporter, core):
    """Two loops on one EPOLLEXCLUSIVE socket: concurrent keep-alive scrapers all get served, and
    the tail stays in the sub-millisecond class (the same bound as test_native_scrape_load_latency)."""
    ex = mock_exporter(backend="mock:gpus=8", interval_s=0.05, http_threads=2)
    r = core.scrape_load("127.0.0.1", ex.port, "/metrics", n_requests=800, concurrency=8)
    lat = sorted(r["latencies_s"])
    assert r["errors"] == 0 and len(lat) == 800
    assert lat[int(0.99 * (len(lat) - 1))] < 0.05


@needs_v6
def test_fleet_view_reads_an_exporter_over_ipv6(mock_exporter):
    """`gpumon top --url [v6]:port` (export/fleet.py over the native client): the bracketed IPv6
    URL reaches the dual-stack listener, the Host header carries the brackets."""
    from gpumon.export import fleet

    ex = mock_exporter(listen_addr="", port=0)
    ex.tick()
    frames, errors = fleet.fetch([f"http://[::1]:{ex.port}/metrics", f"http://127.0.0.1:{ex.port}/metrics"])
    assert not errors and len(frames) == 2
    assert len(fleet.gpu_rows(frames[0])) == 2
