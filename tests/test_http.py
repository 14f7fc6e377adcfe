"""/metrics server: endpoints, keep-alive, gzip, HEAD, errors, concurrency, and latency.

The reference has no scrape endpoint (push-only, /root/reference/gpu.py:145); BASELINE.json's
headline metric is p99 /metrics latency, so the server is tested for correctness under load and
for not tearing responses while the sampler swaps snapshots.
"""

import gzip
import http.client
import math
import socket
import struct
import threading

import pytest

from gpumon.export import promtext


def _get(port, path, headers=None, method="GET"):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    c.request(method, path, headers=headers or {})
    r = c.getresponse()
    body = r.read()
    c.close()
    return r.status, dict(r.getheaders()), body


def _read_request(c):
    """One whole request from a scripted server's socket: the headers, then Content-Length bytes
    of body (a client may send the two in separate segments; closing with the body unread would
    reset the connection under the client's response read)."""
    buf = b""
    while b"\r\n\r\n" not in buf:
        chunk = c.recv(65536)
        if not chunk:
            return
        buf += chunk
    head, _, rest = buf.partition(b"\r\n\r\n")
    n = next((int(l.split(b":", 1)[1]) for l in head.split(b"\r\n") if l.lower().startswith(b"content-length:")), 0)
    while len(rest) < n:
        chunk = c.recv(65536)
        if not chunk:
            return
        rest += chunk


def test_metrics_endpoint(mock_exporter):
    ex = mock_exporter()
    st, h, body = _get(ex.port, "/metrics")
    assert st == 200
    assert h["Content-Type"].startswith("text/plain; version=0.0.4")
    promtext.parse(body.decode())
    assert int(h["Content-Length"]) == len(body)


def test_gzip_negotiation(mock_exporter):
    ex = mock_exporter()
    st, h, body = _get(ex.port, "/metrics", {"Accept-Encoding": "gzip, deflate"})
    assert st == 200 and h.get("Content-Encoding") == "gzip"
    plain = gzip.decompress(body).decode()
    assert plain == ex.metrics_text()
    assert len(body) < len(plain) / 3


def test_gzip_disabled(mock_exporter):
    ex = mock_exporter(gzip=False)
    st, h, body = _get(ex.port, "/metrics", {"Accept-Encoding": "gzip"})
    assert st == 200 and "Content-Encoding" not in h


@pytest.mark.parametrize("during_precompress", [False, True])
def test_concurrent_gzip_scrapes_compress_a_snapshot_once(core, during_precompress):
    """Scrapes that ask a fresh snapshot for gzip at the same instant, or while the tick thread is
    precompressing it: one thread compresses, the others wait for it -- at most 1 ms
    (Snapshot::kGzipWaitNs, ADVICE r5: the wait runs on an HTTP loop) -- and get the same buffer.
    None compresses again; a scrape that lost the claim to a concurrent compression no longer falls
    back to identity while the winner finishes within the wait. A loaded CI host can stretch one
    compression past the wait (then a waiter rightly serves identity), so the race gets 5 attempts;
    the old lost-claim bug failed every attempt."""
    lines = 12000 if during_precompress else 2400  # long enough for scrapes to arrive mid-compression
    body = "".join(f'node_gpu_gpu_util{{gpu_id="{i % 8}",host="n{i}"}} {i * 0.37:.3f}\n' for i in range(lines))
    results = [core.snapshot_gzip_race(body, threads=8, during_precompress=during_precompress) for _ in range(5)]
    # on an overloaded host the scraper threads may start only after the compression in all five:
    # a few more attempts for the mid-compression arrival the precompress case is about
    while during_precompress and not any(r[2] >= 1 for r in results) and len(results) < 20:
        results.append(core.snapshot_gzip_race(body, threads=8, during_precompress=True))
    # whoever got a gzip body got THE one (compressed once), and no waiter stalled past the budget
    assert all(distinct == 1 for gz, distinct, _, _ in results if gz is not None), results
    # the 1 ms budget plus scheduling: a waiter preempted on an oversubscribed host can overrun it,
    # the typical one does not (the old 20 ms wait showed in every attempt)
    waits = sorted(r[3] for r in results)
    assert waits[len(waits) // 2] < 0.005 and waits[-1] < 0.05, waits
    if during_precompress:
        assert any(mid >= 1 for _, _, mid, _ in results)  # the scrapes did arrive while it ran
    else:
        ok = [gz for gz, distinct, _, _ in results if gz is not None and distinct == 1]
        assert ok, [(gz is not None, distinct, mid) for gz, distinct, mid, _ in results]
        assert gzip.decompress(ok[0]).decode() == body


def test_a_long_compression_does_not_stall_the_loop(core):
    """a scrape that finds another thread compressing its snapshot waited up to 20 ms on
    the HTTP loop, stalling every other connection of that loop. It now waits at most 1 ms
    (Snapshot::kGzipWaitNs) and answers with the identity body: a 6 MB body (tens of ms to compress)
    holds no waiter past a few ms."""
    body = "".join(f'node_gpu_gpu_util{{gpu_id="{i % 8}",host="n{i}"}} {i * 0.37:.3f}\n' for i in range(110000))
    runs = [core.snapshot_gzip_race(body, threads=4, during_precompress=True) for _ in range(3)]
    for gz, distinct, mid, longest in runs:
        assert mid >= 1, mid  # the scrapes did arrive while the compression ran
        assert gz is None  # the waiters gave up and served identity
    # the 1 ms budget: the old 20 ms wait showed in every run, a waiter preempted on a loaded host
    # shows in one at most
    assert min(r[3] for r in runs) < 0.008, [r[3] for r in runs]


def test_head_and_404_and_index(mock_exporter):
    ex = mock_exporter()
    st, h, body = _get(ex.port, "/metrics", method="HEAD")
    assert st == 200 and body == b"" and int(h["Content-Length"]) > 0
    assert _get(ex.port, "/nope")[0] == 404
    assert _get(ex.port, "/")[0] == 200
    assert _get(ex.port, "/metrics?x=1")[0] == 200


def test_method_not_allowed(mock_exporter):
    ex = mock_exporter()
    assert _get(ex.port, "/metrics", method="POST")[0] == 405


def test_health_endpoints(mock_exporter):
    ex = mock_exporter()
    assert _get(ex.port, "/healthz")[0] == 200
    assert _get(ex.port, "/readyz")[0] == 200


def test_keepalive_many_requests_one_connection(mock_exporter):
    ex = mock_exporter()
    c = http.client.HTTPConnection("127.0.0.1", ex.port, timeout=5)
    for _ in range(50):
        c.request("GET", "/metrics")
        r = c.getresponse()
        assert r.status == 200
        r.read()
    c.close()


def test_pipelined_requests(mock_exporter):
    ex = mock_exporter()
    s = socket.create_connection(("127.0.0.1", ex.port), timeout=5)
    s.sendall(b"GET /healthz HTTP/1.1\r\nHost: x\r\n\r\nGET /healthz HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
    data = b""
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    s.close()
    assert data.count(b"HTTP/1.1 200 OK") == 2


def test_http10_closes(mock_exporter):
    ex = mock_exporter()
    s = socket.create_connection(("127.0.0.1", ex.port), timeout=5)
    s.sendall(b"GET /healthz HTTP/1.0\r\n\r\n")
    data = b""
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    assert b"Connection: close" in data


def test_bad_request_and_oversized_header(mock_exporter):
    ex = mock_exporter()
    s = socket.create_connection(("127.0.0.1", ex.port), timeout=5)
    s.sendall(b"GARBAGE\r\n\r\n")
    assert b"400" in s.recv(4096)
    s.close()
    s = socket.create_connection(("127.0.0.1", ex.port), timeout=5)
    s.sendall(b"GET /metrics HTTP/1.1\r\nX: " + b"a" * 20000 + b"\r\n\r\n")
    assert b"431" in s.recv(4096)
    s.close()


def test_concurrent_scrapes_while_ticking_no_torn_bodies(mock_exporter, core):
    """Snapshots are immutable: every response body must be one complete, parseable exposition."""
    ex = mock_exporter(backend="mock:gpus=8", interval_s=0.01, http_threads=2)
    errors = []

    def worker():
        c = http.client.HTTPConnection("127.0.0.1", ex.port, timeout=5)
        for _ in range(12):
            c.request("GET", "/metrics")
            r = c.getresponse()
            body = r.read()
            try:
                promtext.parse(body.decode())
                assert body.endswith(b"\n")
            except Exception as e:  # noqa: BLE001
                errors.append(e)
        c.close()

    ts = [threading.Thread(target=worker) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:3]
    assert ex.self_stats()["ticks"] > 5


def test_native_scrape_load_latency(mock_exporter, core):
    ex = mock_exporter(backend="mock:gpus=8", interval_s=0.05)
    r = core.scrape_load("127.0.0.1", ex.port, "/metrics", n_requests=400, concurrency=4)
    lat = sorted(r["latencies_s"])
    assert r["errors"] == 0 and len(lat) == 400
    p99 = lat[int(0.99 * (len(lat) - 1))]
    assert p99 < 0.05, p99  # pre-rendered snapshot: sub-millisecond typical, generous CI bound
    # the server counts a scrape after its last write returns: the client may read the final
    # response a moment before that
    import time
    deadline = time.monotonic() + 5
    while ex.self_stats()["scrapes"] < 400 and time.monotonic() < deadline:
        time.sleep(0.005)
    assert ex.self_stats()["scrapes"] >= 400
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.values(fam, "gpumon_scrape_duration_seconds_count")[0] >= 1


def test_exact_window_quantiles_match_the_recorded_durations(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=2", interval_s=0)
    assert math.isnan(ex.scrape_quantile(0.99))
    ex.tick()
    ex.tick()
    for _ in range(50):
        assert _get(ex.port, "/metrics")[0] == 200
    d = sorted(ex.scrape_durations_since(0))
    assert len(d) == ex.scrape_count() >= 50
    # Nearest-rank quantile over the ring: q=0 is the minimum, q=1 the maximum, q=0.5 the
    # ceil(n/2)-th smallest. float32 ring, so compare at float precision.
    assert ex.scrape_quantile(0.0) == pytest.approx(d[0], rel=1e-6)
    assert ex.scrape_quantile(1.0) == pytest.approx(d[-1], rel=1e-6)
    assert ex.scrape_quantile(0.5) == pytest.approx(d[math.ceil(0.5 * len(d)) - 1], rel=1e-6)
    s50, s100 = ex.sample_quantile(0.5), ex.sample_quantile(1.0)
    assert 0 < s50 <= s100


def test_port_conflict_reports_error(core):
    """One listening socket per server and no SO_REUSEPORT: a second exporter on a taken port fails
    with EADDRINUSE instead of sharing the scrapes (tests/test_listen.py covers both entry points)."""
    a = core.Exporter({"backend": "mock", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0})
    a.start()
    try:
        b = core.Exporter({"backend": "mock", "listen_addr": "127.0.0.1", "port": a.port, "interval_s": 0})
        with pytest.raises(RuntimeError, match="Address already in use"):
            b.start()
        b.stop()
    finally:
        a.stop()


def test_client_refuses_huge_content_length_and_reads_bodies_whole(core):
    """The native client sizes its buffer from Content-Length (csrc/core/http_client.cpp): an
    announced body over 256 MiB is refused before any allocation; a short body is an error."""
    import socket
    import threading

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(4)
    port = srv.getsockname()[1]
    answers = [b"HTTP/1.1 200 OK\r\nContent-Length: 1000000000000\r\n\r\nabc",
               b"HTTP/1.1 200 OK\r\nContent-Length: 10\r\nConnection: close\r\n\r\nabc",
               b"HTTP/1.1 200 OK\r\nContent-Length: 300000\r\nConnection: close\r\n\r\n" + b"x" * 300000]

    def serve():
        for a in answers:
            c, _ = srv.accept()
            c.recv(4096)
            c.sendall(a)
            c.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    st, body, err = core.http_request("GET", f"http://127.0.0.1:{port}/", "", "", 5.0)
    assert st != 200 and "refused" in err
    st, body, err = core.http_request("GET", f"http://127.0.0.1:{port}/", "", "", 5.0)
    assert st != 200 and "short body" in err
    st, body, err = core.http_request("GET", f"http://127.0.0.1:{port}/", "", "", 5.0)
    assert st == 200 and body == b"x" * 300000
    t.join(5)
    srv.close()


@pytest.mark.parametrize("script,error", [
    # a server that drips its header a byte at a time: each recv() returns before SO_RCVTIMEO
    ([b"H"] + [b"x"] * 400, "response timed out"),
    ([b"HTTP/1.1 200 OK\r\nX: " + b"a" * (70 << 10)], "response header too large"),
    # no Content-Length: read to EOF, but the drip never ends
    ([b"HTTP/1.1 200 OK\r\n\r\n"] + [b"y"] * 400, "response timed out"),
    ([b"HTTP/1.1 200 OK\r\nContent-Length: 1000\r\n\r\n"] + [b"z"] * 400, "response timed out"),
])
def test_client_bounds_a_dripping_or_endless_response(core, script, error):
    """The native client (Influx push, csrc/core/http_client.cpp) bounds the whole response by
    twice its timeout and the header by 64 KiB, not just each recv()."""
    import time

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    stop = threading.Event()

    def serve():
        c, _ = srv.accept()
        try:
            _read_request(c)
            for part in script:
                if stop.is_set():
                    break
                c.sendall(part)
                if len(part) < 100:
                    time.sleep(0.01)
        except OSError:
            pass
        finally:
            c.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    t0 = time.monotonic()
    st, body, err = core.http_request("GET", f"http://127.0.0.1:{port}/", "", "", 0.5)
    dt = time.monotonic() - t0
    stop.set()
    t.join(5)
    srv.close()
    assert st == -1 and err == error, (st, err)
    assert dt < 2.5, dt


def test_client_decodes_chunked_bodies_and_keeps_the_connection(core):
    """RFC 9112 chunked responses (a reverse proxy in front of InfluxDB answers errors this way):
    chunks with extensions, trailers, several requests over one keep-alive connection; a broken
    chunk framing is an error, not a hang until the timeout."""
    import time

    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(2)
    port = srv.getsockname()[1]
    good = [b"HTTP/1.1 400 Bad Request\r\nTransfer-Encoding: chunked\r\n\r\n"
            b"7;ext=1\r\n{\"code\"\r\n9\r\n:\"invalid\r\n2\r\n\"}\r\n0\r\nX-Trailer: t\r\n\r\n",
            b"HTTP/1.1 200 OK\r\nTransfer-Encoding: Chunked\r\n\r\n3\r\nabc\r\n0\r\n\r\n",
            b"HTTP/1.1 204 No Content\r\n\r\n"]
    conns = []

    def serve():
        c, _ = srv.accept()
        conns.append(c)
        for a in good:  # three answers on ONE connection, a byte-split one in the middle
            _read_request(c)
            if a is good[1]:
                for i in range(len(a)):
                    c.sendall(a[i:i + 1])
            else:
                c.sendall(a)
        c2, _ = srv.accept()  # then a connection with a broken chunk (size says 5, 3 bytes + CRLF)
        conns.append(c2)
        _read_request(c2)
        c2.sendall(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nabc\r\n0\r\n\r\n")
        time.sleep(0.5)
        c2.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    st, body, err = core.http_request("POST", f"http://127.0.0.1:{port}/write", "m v=1", "", 2.0, "", False, 3)
    assert st == 204, err  # the third answer, over the same connection (the server accepted once)
    t0 = time.monotonic()
    st, body, err = core.http_request("GET", f"http://127.0.0.1:{port}/", "", "", 2.0)
    assert st == -1 and "bad chunked body" in err, (st, err)
    assert time.monotonic() - t0 < 3
    t.join(5)
    srv.close()
    for c in conns:
        c.close()


def test_client_returns_a_chunked_error_body(core):
    """The first chunked answer's body, decoded (what the pusher logs for a 4xx)."""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def serve():
        c, _ = srv.accept()
        _read_request(c)
        c.sendall(b"HTTP/1.1 400 Bad Request\r\nTransfer-Encoding: chunked\r\nConnection: close\r\n\r\n"
                  b"6\r\nfield \r\n7\r\ninvalid\r\n0\r\n\r\n")
        c.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    st, body, err = core.http_request("POST", f"http://127.0.0.1:{port}/write", "m v=1", "", 2.0)
    t.join(5)
    srv.close()
    assert (st, body) == (400, b"field invalid"), (st, body, err)


def test_per_request_family_filter(mock_exporter):
    """/metrics?include=&exclude= (shell globs, comma-separated, repeatable, percent-decoded): the
    same families the config filter would keep, cut from the current snapshot, gzip included; other
    query parameters leave the body untouched."""
    ex = mock_exporter(backend="mock:gpus=2")
    ex.tick()
    full = promtext.parse(ex.metrics_text())
    st, _, body = _get(ex.port, "/metrics?exclude=gpu_xcd_*,gpumon_scrape_duration_seconds")
    fam = promtext.parse(body.decode())
    assert st == 200
    assert set(fam) == set(full) - {n for n in full if n.startswith("gpu_xcd_")} - {"gpumon_scrape_duration_seconds"}
    assert "gpumon_scrape_duration_seconds_bucket" not in body.decode()  # histogram lines go with it
    st, h, body = _get(ex.port, "/metrics?include=node_gpu_%2A&include=gpu_up&exclude=node_gpu_mem_bw_util",
                       {"Accept-Encoding": "gzip"})
    assert st == 200 and h.get("Content-Encoding") == "gzip"
    fam = promtext.parse(gzip.decompress(body).decode())
    assert set(fam) == {n for n in full if n.startswith("node_gpu_") and n != "node_gpu_mem_bw_util"} | {"gpu_up"}
    for _ in range(3):  # cached per snapshot: repeated requests agree
        assert promtext.parse(_get(ex.port, "/metrics?include=gpu_up")[2].decode()).keys() == {"gpu_up"}
    st, _, body = _get(ex.port, "/metrics?foo=bar")
    assert st == 200 and set(promtext.parse(body.decode())) >= set(full) - {"gpumon_scrape_duration_seconds"}


def test_glob_match_agrees_with_fnmatch(core):
    """The native family-filter glob (render.cpp glob_match) follows shell-glob rules: same answers
    as Python's fnmatchcase on '*', '?' and bracket classes, over random patterns and names."""
    import fnmatch
    import random

    rnd = random.Random(4)
    alphabet = "ab_"
    atoms = ["*", "?", "a", "b", "_", "[ab]", "[!a]", "[a-b]", "**"]
    names = ["".join(rnd.choice(alphabet) for _ in range(rnd.randint(0, 8))) for _ in range(60)]
    names += ["gpu_xcd_busy_percent", "node_gpu_gpu_util", "gpumon_scrape_duration_seconds"]
    pats = ["".join(rnd.choice(atoms) for _ in range(rnd.randint(0, 6))) for _ in range(300)]
    pats += ["gpu_xcd_*", "node_gpu_*", "*_seconds", "gpu_?cd_*", "[gn]*_util", "*"]
    bad = [(p, n) for p in pats for n in names if core.glob_match(p, n) != fnmatch.fnmatchcase(n, p)]
    assert not bad, bad[:10]


def test_pathological_filter_is_fast_and_oversized_filters_are_refused(mock_exporter):
    """a '*a*a*a...*b' glob made glibc fnmatch backtrack exponentially on the HTTP loop.
    The native matcher is linear in the name per star position; the longest allowed glob against
    every family stays in milliseconds, and over-long / too many globs get a 400."""
    import time

    ex = mock_exporter(backend="mock:gpus=8")
    ex.tick()
    glob = ("*a" * 63) + "*b"  # 128 bytes, the per-glob limit
    q = "include=" + ",".join([glob] * 32)  # 32 globs, the count limit ('*' needs no escaping)
    t0 = time.perf_counter()
    st, _, body = _get(ex.port, "/metrics?" + q)
    assert st == 200 and time.perf_counter() - t0 < 1.0
    st, _, body = _get(ex.port, "/metrics?include=" + "a" * 129)
    assert st == 400 and b"glob longer than 128" in body
    st, _, body = _get(ex.port, "/metrics?include=" + ",".join(["x*"] * 33))
    assert st == 400 and b"more than 32 globs" in body
    st, _, body = _get(ex.port, "/metrics?exclude=" + "x," * 4100)
    assert st == 400 and b"query longer than" in body
    st, _, _ = _get(ex.port, "/metrics?include=gpu_up")  # the loop is still serving
    assert st == 200


def test_http_rt_loops_are_budget_capped(core):
    """http_rt_priority: the HTTP loops run SCHED_FIFO (where CAP_SYS_NICE allows), and under an
    unthrottled flood each loop drops to normal scheduling once it used its budget of the 100 ms
    window (profiles/r4_scrape_contention.md), so the flood cannot hold a CPU at RT priority."""
    import os

    ex = core.Exporter({"backend": "mock:gpus=2", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0.1,
                        "http_threads": 2, "http_rt_priority": 1, "http_rt_budget": 0.05})
    assert ex.start() == ""
    try:
        ex.wait_for_seq(1, 10)
        st = ex.self_stats()
        try:
            os.sched_setscheduler(0, os.SCHED_FIFO, os.sched_param(1))
            os.sched_setscheduler(0, os.SCHED_OTHER, os.sched_param(0))
        except PermissionError:
            assert st["http_rt_loops"] == 0  # no CAP_SYS_NICE: normal scheduling, said so
            return
        import time

        deadline = time.time() + 5  # each loop thread switches itself to FIFO when it starts
        while ex.self_stats()["http_rt_loops"] < 2 and time.time() < deadline:
            time.sleep(0.02)
        st = ex.self_stats()
        assert st["http_rt_loops"] == 2 and st["http_rt_demotions"] == 0
        r = core.scrape_load("127.0.0.1", ex.port, "/metrics", n_requests=0, duration_s=1.5, concurrency=4,
                             rate_hz=0.0, keep_alive=True, gzip=False)
        assert r["errors"] == 0 and len(r["latencies_s"]) > 100
        assert ex.self_stats()["http_rt_demotions"] > 0
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpumon_http_rt_demotions_total") > 0
    finally:
        ex.stop()


def test_slow_reader_gets_whole_pipelined_bodies_and_a_vanishing_one_is_dropped(mock_exporter, monkeypatch):
    """A scraper that reads slower than the exposition is written: with a small send buffer the
    server's writev() hits EAGAIN mid-body, parks the connection on EPOLLOUT and resumes; the
    pipelined requests behind it are answered in order once it drains. A client that hangs up
    mid-body costs only its own connection."""
    import time

    monkeypatch.setenv("GPUMON_HTTP_SNDBUF", "4096")
    ex = mock_exporter(backend="mock:gpus=8", interval_s=0, gzip=False)
    ex.tick()
    want = ex.metrics_text().encode()
    assert len(want) > 50_000
    s = socket.create_connection(("127.0.0.1", ex.port))
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
    s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n" * 3)
    time.sleep(0.3)  # the server fills both buffers and waits
    buf = b""
    bodies = []
    s.settimeout(5)
    while len(bodies) < 3:
        while b"\r\n\r\n" not in buf:
            buf += s.recv(1 << 16)
        head, _, buf = buf.partition(b"\r\n\r\n")
        assert head.startswith(b"HTTP/1.1 200")
        n = int(next(h for h in head.split(b"\r\n") if h.lower().startswith(b"content-length:")).split(b":")[1])
        while len(buf) < n:
            buf += s.recv(1 << 16)
        bodies.append(buf[:n])
        buf = buf[n:]
        time.sleep(0.05)
    s.close()
    assert bodies == [want] * 3
    # hang up with a body half-written
    s = socket.create_connection(("127.0.0.1", ex.port))
    s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
    s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n\r\n")
    s.recv(1000)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))  # RST
    s.close()
    time.sleep(0.1)
    assert _get(ex.port, "/metrics")[0] == 200


def test_bad_listen_address_is_reported_and_cleaned_up(core):
    """A start() that fails at the listen address has already brought the backend and its device
    workers up: stop() (and the destructor) must take them down, or the worker threads outlive
    the exporter (a crash at interpreter exit)."""
    import gc
    import os
    import time

    def threads():
        return len(os.listdir("/proc/self/task"))

    # threads of earlier tests in this worker (server / sink daemons) may still be exiting
    base, deadline = threads(), time.time() + 5
    while time.time() < deadline:
        time.sleep(0.2)
        if threads() == base:
            break
        base = threads()
    ex = core.Exporter({"backend": "mock:gpus=4", "listen_addr": "not-an-address", "port": 0, "interval_s": 0,
                        "http_threads": 2})
    with pytest.raises(RuntimeError, match="bad listen address not-an-address"):
        ex.start()
    assert threads() >= base + 4  # one device worker per GPU is running
    ex.stop()
    ex.stop()  # idempotent
    assert threads() <= base
    ex = core.Exporter({"backend": "mock:gpus=4", "listen_addr": "not-an-address", "port": 0, "interval_s": 0})
    with pytest.raises(RuntimeError):
        ex.start()
    del ex  # the destructor alone
    gc.collect()
    deadline = time.time() + 5
    while threads() > base and time.time() < deadline:
        time.sleep(0.01)
    assert threads() <= base


def _raw_exchange(port, data):
    s = socket.create_connection(("127.0.0.1", port), timeout=5)
    s.sendall(data)
    out = b""
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        out += chunk
    s.close()
    return out


def test_request_bodies_are_skipped_bounded_and_validated(mock_exporter):
    ex = mock_exporter()
    # a small body is skipped and the pipelined request behind it is answered
    out = _raw_exchange(ex.port, b"GET /healthz HTTP/1.1\r\nContent-Length: 5\r\n\r\nhello"
                                 b"GET /healthz HTTP/1.1\r\nConnection: close\r\n\r\n")
    assert out.count(b"HTTP/1.1 200 OK") == 2, out
    # a POST with a body: 405, and the body is not read as a request
    out = _raw_exchange(ex.port, b"POST /metrics HTTP/1.1\r\nContent-Length: 4\r\n\r\nGET ")
    assert out.startswith(b"HTTP/1.1 405") and out.count(b"HTTP/1.1") == 1, out
    # an announced body larger than any route takes is refused at once, not buffered
    out = _raw_exchange(ex.port, b"POST /metrics HTTP/1.1\r\nContent-Length: 1000000000000\r\n\r\nxxxx")
    assert out.startswith(b"HTTP/1.1 413"), out
    for bad in (b"-1", b"abc", b"12x", b""):
        out = _raw_exchange(ex.port, b"GET /metrics HTTP/1.1\r\nContent-Length: " + bad + b"\r\n\r\n")
        assert out.startswith(b"HTTP/1.1 400"), (bad, out)
    assert _get(ex.port, "/metrics")[0] == 200


def test_error_answer_survives_a_client_still_sending(mock_exporter):
    """A 413 goes out while the client is still sending the refused body. Closing with unread
    input would RST the connection and the client could lose the answer; the server half-closes
    and drains instead (kLingerNs): the client's further sends succeed, and it reads the 413 and
    then EOF (RFC 7230 6.6)."""
    import time

    ex = mock_exporter()
    s = socket.create_connection(("127.0.0.1", ex.port), timeout=5)
    s.sendall(b"POST /metrics HTTP/1.1\r\nContent-Length: 1000000000\r\n\r\n")
    time.sleep(0.1)  # answered and half-closed by now
    s.sendall(b"x" * 200_000)  # the body keeps coming
    time.sleep(0.1)
    s.sendall(b"x" * 1000)  # a RST by now would fail this send (EPIPE / ECONNRESET)
    s.shutdown(socket.SHUT_WR)
    out = b""
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        out += chunk
    s.close()
    assert out.startswith(b"HTTP/1.1 413 Payload Too Large"), out
    assert b"Connection: close" in out


def test_connection_flood_under_a_low_fd_limit(tmp_path):
    """bin/gpumon-exporter with RLIMIT_NOFILE 64 and 300 idle connections opened against it: the
    connection cap is derived from the limit (fds stay for the sampler), excess connections are
    closed, the sampler keeps ticking, the HTTP loops do not spin on a readable listening socket,
    and /metrics answers once the flood is gone."""
    import os
    import resource
    import subprocess
    import time
    import urllib.request

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()

    def low_limit():
        resource.setrlimit(resource.RLIMIT_NOFILE, (64, 64))

    p = subprocess.Popen([os.path.join(root, "bin", "gpumon-exporter"), "--backend", "mock:gpus=2", "--interval",
                          "0.05", "--listen", f"127.0.0.1:{port}", "--http-threads", "2", "--log-level", "error"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, preexec_fn=low_limit)
    conns = []
    try:
        deadline = time.time() + 20
        while time.time() < deadline:
            try:
                urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=1).read()
                break
            except OSError:
                time.sleep(0.05)

        def cpu_s():
            f = open(f"/proc/{p.pid}/stat").read().rsplit(")", 1)[1].split()
            return (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK")

        def ticks():
            body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
            return promtext.one(promtext.parse(body), "gpumon_ticks_total")

        for _ in range(300):
            c = socket.socket()
            c.settimeout(2)
            try:
                c.connect(("127.0.0.1", port))
                conns.append(c)
            except OSError:
                c.close()
        # a new scraper still gets in while the flood holds every slot: the least recently
        # active idle connection makes room
        urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read()
        time.sleep(0.2)  # the counter is in the exposition from the next tick on
        body = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
        assert promtext.one(promtext.parse(body), "gpumon_http_connections_evicted_total") >= 1
        c0, t0 = cpu_s(), time.time()
        time.sleep(1.5)
        burn = (cpu_s() - c0) / (time.time() - t0)
        open_fds = len(os.listdir(f"/proc/{p.pid}/fd"))
        assert p.poll() is None
        assert open_fds <= 64, open_fds
        assert burn < 0.5, burn  # a spinning loop would burn a whole CPU
        for c in conns:
            c.close()
        conns.clear()
        time.sleep(0.3)
        t1 = ticks()
        time.sleep(0.3)
        assert ticks() > t1  # still sampling, and /metrics answers
    finally:
        for c in conns:
            c.close()
        p.terminate()  # also when an assertion above failed: no exporter left behind
        p.wait(10)


def test_flood_evicts_fresh_connections_before_the_scrapers_keep_alive(tmp_path):
    """at the connection cap, eviction prefers connections that never completed a
    request (idle ones, then ones holding a partial request) over a keep-alive connection that has
    served scrapes, which sits idle between them. Prometheus keeps its connection through a connect
    flood. One HTTP loop, RLIMIT_NOFILE 64: a cap of a few dozen connections."""
    import http.client
    import os
    import resource
    import subprocess
    import time
    import urllib.request

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()

    def low_limit():
        resource.setrlimit(resource.RLIMIT_NOFILE, (64, 64))

    p = subprocess.Popen([os.path.join(root, "bin", "gpumon-exporter"), "--backend", "mock:gpus=1", "--interval",
                          "0.1", "--listen", f"127.0.0.1:{port}", "--http-threads", "1", "--log-level", "error"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, preexec_fn=low_limit)
    flood = []
    try:
        deadline = time.time() + 20
        while time.time() < deadline:
            try:
                urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=1).read()
                break
            except OSError:
                time.sleep(0.05)
        scraper = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
        scraper.request("GET", "/metrics")
        assert scraper.getresponse().read()
        local = scraper.sock.getsockname()
        # trickling requests first (partial header), then idle sockets, 200 in all: far past the cap
        for k in range(200):
            c = socket.socket()
            c.settimeout(2)
            try:
                c.connect(("127.0.0.1", port))
                if k < 20:
                    c.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n")  # no blank line: partial
                flood.append(c)
            except OSError:
                c.close()
            time.sleep(0.002)
        for _ in range(3):  # the scraper's keep-alive connection survived the flood
            scraper.request("GET", "/metrics")
            r = scraper.getresponse()
            assert r.status == 200 and r.read()
        assert scraper.sock.getsockname() == local  # the same TCP connection, not a reconnect
        # the tricklers (partial requests) outlived some of the idle sockets that came after them
        alive_partial = 0
        for c in flood[:20]:
            c.setblocking(False)
            try:
                alive_partial += c.recv(1) != b""
            except BlockingIOError:
                alive_partial += 1
            except OSError:
                pass
        assert alive_partial > 0
    finally:
        for c in flood:
            c.close()
        p.terminate()
        p.wait(10)


def test_trickled_header_is_dropped(monkeypatch, mock_exporter):
    """A client that sends part of a request header and then nothing is closed after the header
    timeout (GPUMON_HTTP_HEADER_TIMEOUT_S here; 10 s by default), not after the 60 s idle timeout."""
    import time

    monkeypatch.setenv("GPUMON_HTTP_HEADER_TIMEOUT_S", "0.5")
    ex = mock_exporter()
    s = socket.create_connection(("127.0.0.1", ex.port), timeout=10)
    s.sendall(b"GET /metrics HTTP/1.1\r\nHost: x\r\n")  # no blank line: the header never ends
    t0 = time.monotonic()
    assert s.recv(100) == b""  # closed by the server
    assert time.monotonic() - t0 < 5
    s.close()
    # an idle keep-alive connection with nothing pending is not affected
    k = socket.create_connection(("127.0.0.1", ex.port), timeout=10)
    time.sleep(2.2)
    k.sendall(b"GET /healthz HTTP/1.1\r\nHost: x\r\n\r\n")
    assert k.recv(100).startswith(b"HTTP/1.1 200")
    k.close()


def test_gzip_is_lazy_until_scrapes_keep_asking_for_it(mock_exporter):
    """The snapshot is compressed at most once: by the first gzip scrape (lazy) while gzip scrapes
    are rare, by the tick thread (eager, off the sample-to-export path) once 4 of the last 8
    snapshots were scraped with gzip. A 1 Hz exporter scraped every 15 s compresses 1 tick in 15
    (gzip was 2/3 of the tick thread's CPU at 8 GPUs, profiles/r5_cpu_8dev.md)."""
    import gzip
    import urllib.request

    ex = mock_exporter(backend="mock:gpus=2", interval_s=0)

    identity = []

    def gz_scrape():
        req = urllib.request.Request(f"http://127.0.0.1:{ex.port}/metrics", headers={"Accept-Encoding": "gzip"})
        with urllib.request.urlopen(req, timeout=5) as r:
            if r.headers.get("Content-Encoding") != "gzip":
                # a scrape that found the tick thread still compressing after 1 ms (a loaded host)
                # gets the identity body instead of stalling the loop (Snapshot::kGzipWaitNs)
                identity.append(1)
                return r.read()
            return gzip.decompress(r.read())

    for _ in range(10):
        ex.tick()
    st = ex.self_stats()
    assert st["gzip_eager"] == 0 and st["gzip_lazy"] == 0  # nobody asked: nothing compressed
    body = gz_scrape()
    assert body == ex.metrics_text().encode()
    gz_scrape()  # same snapshot: compressed once
    assert ex.self_stats()["gzip_lazy"] == 1
    for _ in range(6):  # a gzip scrape per tick
        ex.tick()
        gz_scrape()
    st = ex.self_stats()
    assert st["gzip_eager"] >= 2 and st["gzip_lazy"] == 4, st
    lazy = st["gzip_lazy"]
    for _ in range(4):
        ex.tick()
        gz_scrape()
    assert ex.self_stats()["gzip_lazy"] == lazy  # eager now: scrapes find it compressed
    for _ in range(12):  # scrapes stop: eager stops within a few ticks, unused ones counted
        ex.tick()
    e0 = ex.self_stats()["gzip_eager"]
    for _ in range(5):
        ex.tick()
    st = ex.self_stats()
    assert st["gzip_eager"] == e0 and st["gzip_unused"] >= 1


def test_periodic_gzip_scraper_gets_precompressed_snapshots(mock_exporter):
    """A gzip scraper slower than the sampler (Prometheus every 15 s on a 1 Hz exporter; here every
    6th tick at 20 Hz): the tick thread learns its cadence and compresses the snapshot its next
    scrape will read (mode "predicted"), so that scrape does not compress in line, and the
    snapshots between scrapes are not compressed at all."""
    import gzip
    import time
    import urllib.request

    ex = mock_exporter(backend="mock:gpus=4", interval_s=0.05)

    identity = []

    def gz_scrape():
        req = urllib.request.Request(f"http://127.0.0.1:{ex.port}/metrics", headers={"Accept-Encoding": "gzip"})
        with urllib.request.urlopen(req, timeout=5) as r:
            if r.headers.get("Content-Encoding") != "gzip":
                # a scrape that found the tick thread still compressing after 1 ms (a loaded host)
                # gets the identity body instead of stalling the loop (Snapshot::kGzipWaitNs)
                identity.append(1)
                return r.read()
            return gzip.decompress(r.read())

    t0 = time.monotonic()
    for k in range(4):  # learn the cadence
        time.sleep(max(0.0, t0 + 0.3 * (k + 1) - time.monotonic()))
        gz_scrape()
    s0 = ex.self_stats()
    for k in range(4, 16):
        time.sleep(max(0.0, t0 + 0.3 * (k + 1) - time.monotonic()))
        assert b"node_gpu_gpu_util{" in gz_scrape()
    s1 = ex.self_stats()
    predicted = s1["gzip_predicted"] - s0["gzip_predicted"]
    lazy = s1["gzip_lazy"] - s0["gzip_lazy"]
    ticks = s1["ticks"] - s0["ticks"]
    assert ticks >= 60
    # (a loaded CI host jitters the scrapes: some land a tick off the prediction and compress lazily)
    assert predicted >= 4 and lazy < 12, (predicted, lazy)
    assert predicted + lazy + (s1["gzip_eager"] - s0["gzip_eager"]) <= ticks // 2  # far from one per tick
    assert len(identity) <= 3, len(identity)



@pytest.mark.parametrize("tls", [False, True])
def test_connection_cap_fits_the_memory_limit(core, monkeypatch, tmp_path, tls):
    """with a 256 MiB memory limit (the DaemonSet's, the systemd unit's MemoryMax) and a
    high fd limit, the cap must be low enough that every admitted connection buffering a maximal
    request (~88 KiB, +64 KiB for a TLS session) fits in the limit less 96 MiB for the rest."""
    import subprocess

    monkeypatch.setenv("GPUMON_HTTP_MEMORY_BUDGET", str(256 << 20))
    cfg = {"backend": "mock:gpus=1", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0, "http_threads": 2}
    if tls:
        subprocess.run(["openssl", "req", "-x509", "-newkey", "ec", "-pkeyopt", "ec_paramgen_curve:prime256v1",
                        "-nodes", "-days", "1", "-keyout", str(tmp_path / "k"), "-out", str(tmp_path / "c"),
                        "-subj", "/CN=x"], check=True, capture_output=True, timeout=60)
        cfg.update(tls_cert_file=str(tmp_path / "c"), tls_key_file=str(tmp_path / "k"))
    ex = core.Exporter(cfg)
    assert ex.start() == ""
    try:
        cap = ex.self_stats()["http_max_conns"]
        per = (16 + 64 + 4) * 1024 + 4096 + (64 * 1024 if tls else 0)
        assert cap * per <= (256 - 96) << 20, cap
        assert cap >= (1000 if tls else 1800), cap  # and not needlessly low
    finally:
        ex.stop()


def test_memory_limit_walks_the_cgroup_tree(core, monkeypatch, tmp_path):
    """The limit is the smallest memory.max from the process's cgroup (v2) up to the root -- a pod's
    limit sits on the pod's cgroup, above the container's "max" -- else the v1 controller's limit;
    "max" and v1's page-rounded "unlimited" mean none."""
    monkeypatch.delenv("GPUMON_HTTP_MEMORY_BUDGET", raising=False)
    root = tmp_path / "cg"
    leaf = root / "kubepods.slice" / "pod1.slice" / "cri-abc.scope"
    leaf.mkdir(parents=True)
    (root / "kubepods.slice" / "memory.max").write_text("8589934592\n")
    (root / "kubepods.slice" / "pod1.slice" / "memory.max").write_text("268435456\n")
    (leaf / "memory.max").write_text("max\n")
    cg = tmp_path / "cgroup"
    cg.write_text("0::/kubepods.slice/pod1.slice/cri-abc.scope\n")
    assert core.memory_limit_bytes(str(cg), str(root)) == 256 << 20
    (leaf / "memory.max").write_text("134217728\n")  # a tighter container limit wins
    assert core.memory_limit_bytes(str(cg), str(root)) == 128 << 20
    # cgroup v1: no "0::" line, the memory controller's limit file
    v1 = tmp_path / "v1"
    (v1 / "memory").mkdir(parents=True)
    (v1 / "memory" / "memory.limit_in_bytes").write_text("536870912\n")
    cg.write_text("12:memory:/kubepods/pod1/abc\n")
    assert core.memory_limit_bytes(str(cg), str(v1)) == 512 << 20
    (v1 / "memory" / "memory.limit_in_bytes").write_text("9223372036854771712\n")  # unlimited
    assert core.memory_limit_bytes(str(cg), str(v1)) == 0
    assert core.memory_limit_bytes(str(tmp_path / "none"), str(tmp_path / "none")) == 0
    monkeypatch.setenv("GPUMON_HTTP_MEMORY_BUDGET", "1000")
    assert core.memory_limit_bytes(str(cg), str(root)) == 1000
