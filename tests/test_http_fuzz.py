"""Hypothesis fuzzing of the epoll HTTP server with raw bytes (the scrape endpoint faces every
pod on the node network). Whatever arrives -- garbage, truncated or pipelined requests, huge
headers, odd methods -- the server must answer with a well-formed HTTP/1.1 status line or close
the connection, and keep serving /metrics afterwards."""

import socket

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

methods = st.sampled_from(["GET", "HEAD", "POST", "PUT", "DELETE", "OPTIONS", "G\x00T", "", "get"])
paths = st.sampled_from(["/metrics", "/", "/healthz", "/readyz", "/livez", "/nope", "*", "", "/metrics?x=1",
                         "/" + "a" * 5000])
versions = st.sampled_from(["HTTP/1.1", "HTTP/1.0", "HTTP/2.0", "HTTP/9", ""])
header_line = st.tuples(st.text(alphabet="abcdefghijklmnopqrstuvwxyz-", min_size=0, max_size=20),
                        st.text(alphabet=st.characters(min_codepoint=32, max_codepoint=126), max_size=60))
request = st.builds(
    lambda m, p, v, hs, tail, crlf: (f"{m} {p} {v}" + crlf + "".join(f"{k}: {val}{crlf}" for k, val in hs) + crlf
                                     ).encode("latin-1", "replace") + tail,
    methods, paths, versions, st.lists(header_line, max_size=6), st.binary(max_size=64),
    st.sampled_from(["\r\n", "\n"]))
payload = st.one_of(request, st.binary(min_size=1, max_size=2048), st.lists(request, min_size=2, max_size=4).map(b"".join))


@pytest.fixture(scope="module")
def server():
    from gpumon import core as _core

    core = _core()
    ex = core.Exporter({"backend": "mock:gpus=2", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                        "http_threads": 2})
    ex.start()
    ex.tick()
    yield ex
    ex.stop()


def _exchange(port, data, timeout=2.0):
    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
    try:
        s.sendall(data)
        s.shutdown(socket.SHUT_WR)
        out = b""
        while True:
            try:
                chunk = s.recv(65536)
            except socket.timeout:
                break
            if not chunk:
                break
            out += chunk
        return out
    finally:
        s.close()


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(data=payload)
def test_any_bytes_get_a_status_line_or_close(server, data):
    out = _exchange(server.port, data)
    if out:
        assert out.startswith(b"HTTP/1.1 "), out[:80]
        code = int(out[9:12])
        assert code in (200, 400, 404, 405, 431, 505), out[:80]
    # the server is still healthy
    ok = _exchange(server.port, b"GET /healthz HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
    assert ok.startswith(b"HTTP/1.1 200"), ok[:80]


@pytest.mark.slow
def test_asan_build_survives_raw_fuzz():
    """The same kind of inputs against the ASan/UBSan build of the native exporter: any memory error
    in the request parser aborts the process and fails here."""
    import os
    import random
    import subprocess
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    from conftest import make_locked

    r = make_locked("asan", jobs=8)
    assert r.returncode == 0, r.stderr[-2000:]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.Popen([os.path.join(root, "bin/gpumon-exporter-asan"), "--backend", "mock:gpus=2",
                          "--interval", "0.05", "--listen", f"127.0.0.1:{port}", "--log-level", "error"],
                         stderr=subprocess.PIPE, stdout=subprocess.DEVNULL, env=env, text=True)
    try:
        deadline = time.time() + 30
        while time.time() < deadline:
            try:
                if _exchange(port, b"GET /healthz HTTP/1.1\r\n\r\n").startswith(b"HTTP/1.1"):
                    break
            except OSError:
                time.sleep(0.1)
        rng = random.Random(1234)
        seeds = [b"GET /metrics HTTP/1.1\r\nHost: a\r\nAccept-Encoding: gzip\r\n\r\n",
                 b"HEAD / HTTP/1.0\r\n\r\n", b"POST /metrics HTTP/1.1\r\nContent-Length: 5\r\n\r\nhello",
                 b"GET /" + b"x" * 9000 + b" HTTP/1.1\r\n\r\n", b"\r\n\r\n\r\n", b"GET /metrics HTTP/1.1\r\n" * 50]
        for i in range(400):
            base = bytearray(rng.choice(seeds))
            for _ in range(rng.randint(0, 8)):  # random byte flips / truncation / duplication
                op = rng.random()
                if op < 0.4 and base:
                    base[rng.randrange(len(base))] = rng.randrange(256)
                elif op < 0.7:
                    base = base[: rng.randrange(len(base) + 1)]
                else:
                    base += base[: rng.randrange(len(base) + 1)]
            try:
                _exchange(port, bytes(base), timeout=1.0)
            except OSError:
                pass
            assert p.poll() is None, p.stderr.read()[-4000:]
        assert _exchange(port, b"GET /metrics HTTP/1.1\r\nConnection: close\r\n\r\n").startswith(b"HTTP/1.1 200")
    finally:
        p.terminate()
        try:
            err = p.communicate(timeout=10)[1]
        except subprocess.TimeoutExpired:
            p.kill()
            err = p.communicate()[1]
    assert "AddressSanitizer" not in err and "runtime error" not in err, err[-4000:]


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(body=st.binary(max_size=3000), sizes=st.lists(st.integers(min_value=1, max_value=700), min_size=1, max_size=12),
       split=st.integers(min_value=1, max_value=97), ext=st.booleans())
def test_client_chunked_decoding_round_trips(body, sizes, split, ext):
    """The native client's chunked decoder (csrc/core/http_client.cpp) against random chunkings of
    random bodies, delivered in random-sized TCP segments: the decoded body is the original."""
    import threading
    import time

    from gpumon import core as _core

    chunks, i, k = [], 0, 0
    while i < len(body):
        n = sizes[k % len(sizes)]
        chunks.append(body[i:i + n])
        i += n
        k += 1
    wire = b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n"
    for c in chunks:
        wire += f"{len(c):x}{';x=y' if ext else ''}\r\n".encode() + c + b"\r\n"
    wire += b"0\r\n\r\n"
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def serve():
        c, _ = srv.accept()
        c.recv(65536)
        for j in range(0, len(wire), split):
            c.sendall(wire[j:j + split])
        time.sleep(0.05)
        c.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    st_, got, err = _core().http_request("GET", f"http://127.0.0.1:{port}/", "", "", 5.0)
    t.join(5)
    srv.close()
    assert st_ == 200 and got == body, (st_, err, len(got), len(body))
