"""Exposition format: Prometheus text validity, reference-compatible names, escaping, Influx lines.

Reference schema: node_gpu (/root/reference/gpu.py:136-143) and pod_gpu (gpu.py:206-216).
"""

import math
import re

import pytest

from gpumon.export import promtext


def test_prometheus_text_is_valid_and_has_reference_families(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=4")
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    for name in ["node_gpu_gpu_util", "node_gpu_mem_util", "node_gpu_mem_used", "node_gpu_mem_total",
                 "node_gpu_mem_free"]:
        assert name in fam, name
        assert len(fam[name]["samples"]) == 4
        assert fam[name]["type"] == "gauge"
    # labels: host + gpu_id on every device series (reference tags host, gpu_id)
    for _, labels, _ in fam["node_gpu_gpu_util"]["samples"]:
        assert set(labels) == {"host", "gpu_id"}  # the reference's tags (gpu.py:137)
        assert labels["host"] == "node-a"
        assert labels["gpu_id"] in {"0", "1", "2", "3"}
    # identity is carried once per GPU on gpu_info (join on gpu_id)
    for _, labels, _ in fam["gpu_info"]["samples"]:
        assert labels["gpu_uuid"] and labels["bdf"] and labels["gfx_target"] == "gfx950"


def test_full_device_labels_option(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=1", full_device_labels=True)
    fam = promtext.parse(ex.metrics_text())
    _, labels, _ = fam["node_gpu_gpu_util"]["samples"][0]
    assert set(labels) == {"host", "gpu_id", "gpu_uuid", "bdf"}


def test_mem_fields_consistent(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=1")
    fam = promtext.parse(ex.metrics_text())
    total = promtext.one(fam, "node_gpu_mem_total", gpu_id="0")
    used = promtext.one(fam, "node_gpu_mem_used", gpu_id="0")
    free = promtext.one(fam, "node_gpu_mem_free", gpu_id="0")
    util = promtext.one(fam, "node_gpu_mem_util", gpu_id="0")
    assert total == 294896  # MI355X: 288 GiB HBM3E in MiB
    assert used + free == total
    assert util == pytest.approx(used * 100.0 / total, rel=1e-3)
    assert promtext.one(fam, "gpu_vram_total_bytes", gpu_id="0") == total * 1048576


def test_mi355x_families_present(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=1")
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert len(promtext.values(fam, "gpu_xcd_busy_percent")) == 8          # 8 XCDs
    assert len(promtext.values(fam, "gpu_xgmi_link_up")) == 7              # 7 peer links
    assert promtext.values(fam, "gpu_temperature_celsius", sensor="hotspot")
    assert promtext.one(fam, "gpu_power_limit_watts") == 1400
    assert promtext.values(fam, "gpu_energy_joules_total")[0] > 0
    assert fam["gpu_energy_joules_total"]["type"] == "counter"
    assert promtext.one(fam, "gpumon_gpus", state="total") == 1


def test_unsupported_fields_are_omitted_not_zero(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=1,unsupported=temp_hotspot;xcd")
    fam = promtext.parse(ex.metrics_text())
    assert not promtext.values(fam, "gpu_temperature_celsius", sensor="hotspot")
    assert promtext.values(fam, "gpu_temperature_celsius", sensor="mem")
    assert "gpu_xcd_busy_percent" not in fam  # empty families are dropped entirely


def test_label_escaping(core):
    assert core.escape_label_value('a"b\\c\nd') == 'a\\"b\\\\c\\nd'
    assert core.escape_influx_tag("a b,c=d") == "a\\ b\\,c\\=d"
    assert core.escape_influx_tag("") == "-"
    assert core.escape_influx_field_str('x"y\\') == 'x\\"y\\\\'


@pytest.mark.parametrize("v,s", [(0.0, "0"), (42.0, "42"), (1.5, "1.5"), (float("nan"), "NaN"),
                                 (float("inf"), "+Inf"), (-3.0, "-3"), (309220868096.0, "309220868096")])
def test_number_format(core, v, s):
    assert core.format_double(v) == s


def test_influx_node_gpu_line_matches_reference_layout(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=2")
    lines = [l for l in ex.influx_text().splitlines() if l.startswith("node_gpu,")]
    assert len(lines) == 2
    # gpu.py:136-143: node_gpu,host=H,gpu_id=K gpu_util=..,mem_util=..,mem_used=..,mem_total=..,node="H",gid=K,mem_free=..
    pat = re.compile(r'^node_gpu,host=node-a,gpu_id=(\d) gpu_util=[\d.]+,mem_util=[\d.e-]+,mem_used=\d+,'
                     r'mem_total=\d+,node="node-a",gid=\1,mem_free=\d+ \d{19}$')
    for l in lines:
        assert pat.match(l), l


def test_influx_pod_gpu_line_matches_reference_layout(mock_exporter):
    import os

    ex = mock_exporter(backend="mock:gpus=1")
    ex.mock_set_procs([{"pid": os.getpid(), "device": 0, "name": "python train.py", "vram_bytes": 2 ** 30}])
    ex.tick()
    lines = [l for l in ex.influx_text().splitlines() if l.startswith("pod_gpu,")]
    assert len(lines) == 1
    l = lines[0]
    # tags (gpu.py:207-208) then fields (gpu.py:209-216), escaped
    assert re.match(r"^pod_gpu,host=node-a,namespace=-,gpu_id=0,containerid=[-0-9a-f]+,pid_t=\d+,gpu_util_t=[\d.]+,"
                    r"user_name_t=- procressname=\"python train.py\",podname=\"-\",pid=\"\d+\",gpu_id_v=\"0\","
                    r"node=\"node-a\",user_name=\"-\",gpu_util=[\d.]+,used_memory=1024 \d{19}$", l), l


def test_influx_2018_pod_gpu_layout(mock_exporter):
    """img/influxdb.png: pod_gpu columns containerid, gid, gpu, host, namespace, node, pid, pod,
    procressname, used_gpu (MiB)."""
    import os

    ex = mock_exporter(backend="mock:gpus=2", influx_schema=2018)
    ex.mock_set_procs([{"pid": os.getpid(), "device": 1, "name": "python3", "vram_bytes": 15524 * 2 ** 20}])
    ex.tick()
    lines = [l for l in ex.influx_text().splitlines() if l.startswith("pod_gpu,")]
    assert len(lines) == 1, lines
    assert re.match(r"^pod_gpu,host=node-a,namespace=-,gpu=1,containerid=[-0-9a-f]+ gid=1,node=\"node-a\","
                    r"pid=\"\d+\",pod=\"-\",procressname=\"python3\",used_gpu=15524 \d{19}$", lines[0]), lines[0]
    assert sum(l.startswith("node_gpu,") for l in ex.influx_text().splitlines()) == 2  # node_gpu unchanged


def test_no_nan_in_exposition(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=3")
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    for f in fam.values():
        for _, _, v in f["samples"]:
            assert not math.isnan(v)


def test_influx_extended_pod_gpu_carries_per_process_fields(mock_exporter):
    """influx_extended: the reference pod_gpu line plus the per-process numbers it could not measure
    (busy share, CU-equivalents of waves, MFMA utilisation on an exclusive GPU); the plain schema
    stays byte-for-byte the reference's."""
    import os

    procs = [{"pid": os.getpid(), "device": 0, "name": "train", "vram_bytes": 2 ** 30, "kfd_only": True}]
    plain = mock_exporter(backend="mock:gpus=1,mode=idle", sample_threads=0, mock={"procs": procs})
    ext = mock_exporter(backend="mock:gpus=1,mode=idle", sample_threads=0, influx_extended=True,
                        mock={"procs": procs})
    for ex in (plain, ext):
        ex.mock_set_occ_series(0, [128.0])
        ex.set_device_mfma_util({0: 61.5})
        ex.tick()
    (lp,) = [l for l in plain.influx_text().splitlines() if l.startswith("pod_gpu,")]
    (le,) = [l for l in ext.influx_text().splitlines() if l.startswith("pod_gpu,")]
    assert "proc_gfx_util" not in lp and "mfma_util" not in lp
    assert re.search(r",used_memory=1024,proc_gfx_util=100,cu_occupancy=128,mfma_util=61\.5 \d{19}$", le), le


def test_metric_family_filter(mock_exporter):
    """metrics_include / metrics_exclude (shell globs on family names): a deselected family writes
    no HELP / TYPE / sample line; the rest of the body is unchanged."""
    full = promtext.parse(mock_exporter(backend="mock:gpus=2").metrics_text())
    ex = mock_exporter(backend="mock:gpus=2", metrics_exclude=["gpu_xcd_*", "gpumon_scrape_duration_seconds"])
    text = ex.metrics_text()
    fam = promtext.parse(text)
    assert "gpu_xcd_busy_percent" in full and "gpumon_scrape_duration_seconds" in full
    assert not [n for n in fam if n.startswith("gpu_xcd_")]
    assert "gpumon_scrape_duration_seconds" not in text  # histogram: no _bucket / _sum / _count
    assert set(full) - set(fam) == {n for n in full if n.startswith("gpu_xcd_")} | {"gpumon_scrape_duration_seconds"}
    assert fam["node_gpu_gpu_util"]["samples"] == full["node_gpu_gpu_util"]["samples"]
    # include first, then exclude
    ex = mock_exporter(backend="mock:gpus=2", metrics_include=["node_gpu_*", "gpu_up"],
                       metrics_exclude=["node_gpu_mem_bw_util"])
    fam = promtext.parse(ex.metrics_text())
    assert set(fam) == {n for n in full if n.startswith("node_gpu_") and n != "node_gpu_mem_bw_util"} | {"gpu_up"}
    # the Influx sink keeps the reference's fixed layout
    ex = mock_exporter(backend="mock:gpus=1", metrics_include=["gpu_up"])
    assert any(l.startswith("node_gpu,") for l in ex.influx_text().splitlines())
