"""Fleet view (gpumon/export/fleet.py, `gpumon top --url ...`): several running exporters read over
HTTP, rendered as the reference's two Grafana views (per-card gauges, container table) in a
terminal, without opening a GPU."""

import os
import time

from gpumon import cli
from gpumon.export import fleet, promtext


def _node(mock_exporter, host, gpus=2):
    ex = mock_exporter(backend=f"mock:gpus={gpus},mode=load", host=host, ras_every=1)
    ex.set_allocations([{"pod_namespace": "ml", "pod_name": f"{host}-job-0", "container_name": "c", "gpu_index": 0}])
    ex.mock_set_procs([{"pid": os.getpid(), "device": 1, "name": "python3", "vram_bytes": 3 << 30, "queues": 2}])
    ex.mock_add_ecc(1, "umc", ue=2)
    ex.tick()
    time.sleep(0.05)  # a new firmware table: the second tick has an interval (rates)
    ex.tick()
    return ex


def test_gpu_and_pod_rows_from_an_exposition(mock_exporter):
    ex = _node(mock_exporter, "node-a")
    fam = promtext.parse(ex.metrics_text())
    rows = fleet.gpu_rows(fam)
    assert [(r["host"], r["gpu_id"]) for r in rows] == [("node-a", "0"), ("node-a", "1")]
    r1 = rows[1]
    assert r1["up"] == 1 and len(r1["xcd"]) == 8 and r1["vram_total"] > 280 * 2 ** 30
    assert r1["ecc_ue"] == 2 and rows[0]["ecc_ue"] == 0
    pods = fleet.pod_rows(fam)
    assert {p["podname"] for p in pods} >= {"node-a-job-0"}
    assert any(p["pid"] == str(os.getpid()) and p["used_memory_bytes"] == 3 << 30 and p["queues"] == 2 for p in pods)
    # the PCIe interval rate (two ticks: an interval) next to the other device columns
    pcie = {r["gpu_id"]: r["pcie_Bps"] for r in rows}
    assert all(v is not None and v > 0 for v in pcie.values()), pcie
    text = fleet.render([fam])
    assert "PCIe GB/s" in text and f"{pcie['1'] / 1e9:9.2f}" in text


def test_cli_top_over_two_exporters(mock_exporter, capsys):
    a, b = _node(mock_exporter, "node-a"), _node(mock_exporter, "node-b", gpus=3)
    rc = cli.main(["top", "--url", f"127.0.0.1:{a.port}", "--url", f"http://127.0.0.1:{b.port}/metrics",
                   "--iterations", "1"])
    out = capsys.readouterr().out
    assert rc == 0
    gpu_lines = [l for l in out.splitlines() if l.startswith("node-")]
    assert sum(l.startswith("node-a") for l in gpu_lines) >= 2 + 2  # 2 GPUs + pod rows
    assert "node-b-job-0" in out and "ECC-UE" in out
    # SHARING (gpu_active_processes): node-a's GPU 1 runs this process in the mock -> exclusive
    hdr = next(l for l in out.splitlines() if l.startswith("HOST"))
    assert hdr.rstrip().endswith("SHARING")
    a1 = next(l for l in gpu_lines if l.split()[:2] == ["node-a", "1"])
    assert a1.split()[-1] == "exclusive", a1
    assert fleet.sharing_label(None) == "-" and fleet.sharing_label(0) == "idle"
    assert fleet.sharing_label(3.0) == "shared:3"
    assert sum(1 for l in out.splitlines() if l.startswith("node-b") and "/288 " in l) == 3  # GPU rows


def test_unreachable_exporter_is_reported(mock_exporter, capsys):
    a = _node(mock_exporter, "node-a", gpus=1)
    rc = cli.main(["top", "--url", f"127.0.0.1:{a.port}", "--url", "127.0.0.1:9", "--iterations", "1"])
    out = capsys.readouterr().out
    assert rc == 0 and "127.0.0.1:9/metrics:" in out
    assert cli.main(["top", "--url", "127.0.0.1:9", "--iterations", "1"]) == 1


def test_influx_extended_carries_ras_totals(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=1", influx_extended=True, ras_every=1)
    ex.mock_add_ecc(0, "umc", ue=1, ce=5)
    ex.mock_add_ecc(0, "gfx", ce=2)
    ex.tick()
    ex.tick()  # the RAS read runs after a tick is published; the next tick carries it (ras_async)
    (ext,) = [l for l in ex.influx_text().splitlines() if l.startswith("gpu_ext,")]
    assert "ecc_uncorrectable=1" in ext and "ecc_correctable=7" in ext and "retired_pages=0" in ext


def test_fleet_fetch_runs_nodes_in_parallel(core):
    """Four nodes that each hold the request 0.5 s before answering are fetched in about one node's
    time, and frames keep the order of the URLs."""
    import http.server
    import threading
    import time

    class Slow(http.server.BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            time.sleep(0.5)
            body = ("# TYPE node_gpu_gpu_util gauge\n"
                    f'node_gpu_gpu_util{{host="h{self.server.server_address[1]}",gpu_id="0"}} 1\n').encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srvs = [http.server.ThreadingHTTPServer(("127.0.0.1", 0), Slow) for _ in range(4)]
    for s in srvs:
        threading.Thread(target=s.serve_forever, daemon=True).start()
    try:
        from gpumon.export import fleet

        urls = [f"http://127.0.0.1:{s.server_address[1]}/metrics" for s in srvs]
        t0 = time.monotonic()
        frames, errors = fleet.fetch(urls, timeout_s=5)
        dt = time.monotonic() - t0
    finally:
        for s in srvs:
            s.shutdown()
    assert not errors and len(frames) == 4
    assert dt < 1.5, dt
    hosts = [f["node_gpu_gpu_util"]["samples"][0][1]["host"] for f in frames]
    assert hosts == [f"h{s.server_address[1]}" for s in srvs]


def test_local_top_shows_pcie_rate_and_queues():
    """`gpumon top` (local): the per-GPU PCIe interval rate and each row's hardware queue count
    (`-` where KFD's queue list is not readable)."""
    from gpumon.cli import render_top

    st = [{"gpu_id": "0"}]
    f = {"gfx_util": 100.0, "vram_used": 2 ** 30, "vram_total": 2 ** 38, "power_cur": 1300.0,
         "temp_hotspot": 60.0, "gfxclk_cur": 2100.0}
    sm = [{"fields": f, "xcd_busy": [100.0] * 8}]
    rows = [dict(containerid="-", podname="-", namespace="-", user_name="-", pid="7", dev=0,
                 used_memory_bytes=2 ** 30, proc_gfx_util=50.0, cu_occupancy=128.0, queues=3, procname="train"),
            dict(containerid="-", podname="-", namespace="-", user_name="-", pid="8", dev=0,
                 used_memory_bytes=0, proc_gfx_util=float("nan"), cu_occupancy=float("nan"), queues=-1,
                 procname="peer")]
    text = render_top(st, sm, [{"pcie_Bps": 57.2e9}], rows)
    head, gpu = text.splitlines()[:2]
    assert "PCIe GB/s" in head and "57.20" in gpu
    lines = text.splitlines()
    train = next(l for l in lines if l.endswith("train"))
    peer = next(l for l in lines if l.endswith("peer"))
    assert train.split()[-2] == "3" and peer.split()[-2] == "-"
    assert "-" in render_top(st, sm, [{}], [])  # no rate yet (first tick)
    ctx = [{"pid": 7, "dev": 0, "row": True, "why": ""}, {"pid": 99, "dev": 0, "row": False, "why": "empty"}]
    assert render_top(st, sm, [{}], rows, contexts=ctx).splitlines()[-1] == "hidden: pid 99 gpu 0 empty"


def test_influx_extended_carries_interval_rates(mock_exporter):
    """gpu_ext also carries the interval PCIe rate and power (rates.cpp), the values of the tick's
    rates."""
    import time

    import pytest

    ex = mock_exporter(backend="mock:gpus=1,mode=load", influx_extended=True)
    ex.tick()
    time.sleep(0.05)
    ex.tick()
    (ext,) = [l for l in ex.influx_text().splitlines() if l.startswith("gpu_ext,")]
    fields = dict(kv.split("=") for kv in ext.split(" ")[1].split(","))
    r = ex.rates()[0]
    assert float(fields["pcie_bytes_per_s"]) == pytest.approx(r["pcie_Bps"], rel=1e-6)
    assert float(fields["power_interval_w"]) == pytest.approx(r["power_from_energy_w"], rel=1e-6)
