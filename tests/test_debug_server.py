"""The loopback-only JSON introspection server (`debug_listen`, csrc/core/exporter_debug.cpp).

bench.py reads the shipped binary through it (gpumon/export/child.py): the exact tick log, the
per-scrape service times, samples, pod rows and self stats. It carries no authentication, so it
must refuse every non-loopback address, in the library and in the binary. The reference has no
such surface (it printed to stdout, /root/reference/gpu.py:145).
"""

import http.client
import json
import os
import subprocess
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BINARY = os.path.join(ROOT, "bin", "gpumon-exporter")


def _get(port, path, timeout=10, host="127.0.0.1"):
    c = http.client.HTTPConnection(host, port, timeout=timeout)
    try:
        c.request("GET", path)
        r = c.getresponse()
        return r.status, r.getheader("Content-Type"), r.read()
    finally:
        c.close()


@pytest.fixture()
def ex(core):
    procs = [{"pid": 4242, "device": 0, "name": "train", "kfd_only": True, "vram_bytes": 1 << 30, "queues": 2},
             {"pid": 4243, "device": 1, "name": "probe", "kfd_only": True, "vram_bytes": 0, "queues": 0}]
    e = core.Exporter({"backend": "mock", "mock": {"gpus": 2, "procs": procs}, "listen_addr": "127.0.0.1", "port": 0,
                       "interval_s": 0, "debug_listen": "127.0.0.1:0", "host": "node-a"})
    assert e.start() == ""
    yield e
    e.stop()


def test_views_are_json_and_agree_with_the_bindings(ex):
    port = ex.debug_port
    assert port > 0 and port != ex.port
    for _ in range(3):
        ex.tick()
    st, ctype, body = _get(port, "/debug/state")
    assert st == 200 and ctype.startswith("application/json")
    state = json.loads(body)
    assert state["pid"] == os.getpid() and state["seq"] == ex.seq and state["port"] == ex.port
    assert len(state["statics"]) == len(ex.statics())
    assert {"ticks", "overruns", "scrapes", "cpu_seconds"} <= set(state["self"])
    assert len(state["statics"]) == 2

    ticks = json.loads(_get(port, "/debug/ticks")[2])
    assert [t["seq"] for t in ticks][-3:] == [ex.seq - 2, ex.seq - 1, ex.seq]
    assert all(len(t["dev"]) == len(ex.statics()) for t in ticks)
    assert json.loads(_get(port, f"/debug/ticks?since={ex.seq - 1}")[2])[0]["seq"] == ex.seq

    samples = json.loads(_get(port, "/debug/samples")[2])
    assert [s["index"] for s in samples] == list(range(len(ex.samples())))
    for mine, theirs in zip(samples, ex.samples()):
        for k, v in theirs["fields"].items():
            w = mine["fields"][k]
            assert (w is None and v != v) or w == pytest.approx(v), k  # NaN is JSON null

    procs = json.loads(_get(port, "/debug/procs")[2])
    assert procs == ex.debug_view("/debug/procs")
    assert {(p["dev"], str(p["pid"])) for p in procs if p["row"]} == {(r["dev"], r["pid"]) for r in ex.pod_rows()
                                                                       if not r["idle"]}
    assert {(p["dev"], p["pid"]) for p in procs} == {(0, 4242), (1, 4243)}  # (hidden ones: test_occupancy.py)
    rows = json.loads(_get(port, "/debug/rows")[2])
    train = next(r for r in rows if r["pid"] == "4242")
    assert train["queues"] == 2 and train["used_memory_bytes"] == 1 << 30 and train["procname"] == "train"
    assert [(r["dev"], r["pid"]) for r in rows] == [(r["dev"], r["pid"]) for r in ex.pod_rows()]


def test_scrape_durations_are_the_metrics_servers(ex):
    ex.tick()
    n0 = json.loads(_get(ex.debug_port, "/debug/scrapes")[2])["count"]
    for _ in range(5):
        with urllib.request.urlopen(f"http://127.0.0.1:{ex.port}/metrics", timeout=5) as r:
            assert r.status == 200
    # the server stamps a scrape after its write returns, which can be after the client read it
    import time

    deadline = time.time() + 5
    sc = json.loads(_get(ex.debug_port, f"/debug/scrapes?since={n0}")[2])
    while sc["count"] < n0 + 5 and time.time() < deadline:
        time.sleep(0.01)
        sc = json.loads(_get(ex.debug_port, f"/debug/scrapes?since={n0}")[2])
    assert sc["count"] == n0 + 5
    assert len(sc["durations_s"]) == 5 and all(0 < d < 1 for d in sc["durations_s"])
    # the debug server's own requests are not /metrics scrapes
    assert json.loads(_get(ex.debug_port, "/debug/scrapes")[2])["count"] == n0 + 5


def test_wait_returns_at_the_tick_or_the_timeout(ex):
    seq = ex.seq
    w = json.loads(_get(ex.debug_port, f"/debug/wait?seq={seq + 1}&timeout_s=0.2")[2])
    assert w == {"seq": seq, "ok": False}  # interval 0: nothing ticks on its own
    assert json.loads(_get(ex.debug_port, f"/debug/wait?seq={seq}&timeout_s=0")[2])["ok"] is True


def test_unknown_path_is_404_and_metrics_is_not_served(ex):
    assert _get(ex.debug_port, "/debug/nope")[0] == 404
    assert _get(ex.debug_port, "/metrics")[0] == 404


@pytest.mark.parametrize("addr", ["0.0.0.0:0", "[::]:0", "10.1.2.3:9500", ":9500"])
def test_non_loopback_addresses_are_refused(core, addr):
    e = core.Exporter({"backend": "mock", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                       "debug_listen": addr})
    with pytest.raises(RuntimeError, match="loopback addresses only"):
        e.start()
    e.stop()


@pytest.mark.parametrize("addr", ["127.0.0.1:0", "localhost:0", "[::1]:0", "127.0.0.2:0"])
def test_loopback_addresses_are_accepted(core, addr):
    e = core.Exporter({"backend": "mock", "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0,
                       "debug_listen": addr})
    try:
        try:
            e.start()
        except RuntimeError as err:
            if addr.startswith("[::1]") and "assign" in str(err):
                pytest.skip("no IPv6 loopback here")
            raise
        assert e.debug_port > 0
        host = {"localhost:0": "127.0.0.1", "[::1]:0": "::1"}.get(addr, addr.rsplit(":", 1)[0])
        assert _get(e.debug_port, "/debug/state", host=host)[0] == 200
    finally:
        e.stop()


def test_binary_refuses_a_non_loopback_debug_listen(tmp_path):
    if not os.access(BINARY, os.X_OK):
        pytest.skip("bin/gpumon-exporter not built")
    p = subprocess.run([BINARY, "--backend", "mock", "--listen", "127.0.0.1:0", "--debug-listen", "0.0.0.0:9599",
                        "--once"], capture_output=True, text=True, timeout=30)
    assert p.returncode == 2 and "loopback addresses only" in p.stderr, (p.returncode, p.stderr)
