"""The REAL AmdSmiBackend (dlopen table, metrics parsing, N/A handling, resize paths, fallbacks)
exercised on CPU against build/fakes/libfake_amd_smi.so (csrc/fakes/fake_amd_smi.cpp), which
returns MI355X-shaped gpu_metrics v1.8 tables."""

import os

import pytest

from conftest import make_locked
from gpumon.export import promtext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(ROOT, "build", "fakes", "libfake_amd_smi.so")


@pytest.fixture(scope="module", autouse=True)
def fake_lib():
    make_locked("fakes")
    return FAKE


@pytest.fixture
def fake_exporter(core, monkeypatch):
    made = []

    def make(env=None, **over):
        for k in ("FAKE_AMDSMI_GPUS", "FAKE_AMDSMI_PROCS", "FAKE_AMDSMI_FAIL_METRICS", "FAKE_AMDSMI_INIT_FAIL",
                  "FAKE_AMDSMI_NO_METRICS", "FAKE_AMDSMI_UNSUPPORTED", "FAKE_AMDSMI_BUSY",
                  "FAKE_AMDSMI_DRIVER_VERSION"):
            monkeypatch.delenv(k, raising=False)
        for k, v in (env or {}).items():
            monkeypatch.setenv(k, str(v))
        cfg = {"backend": "amdsmi", "amdsmi_lib": FAKE, "serve_http": False, "interval_s": 0, "host": "n1",
               "verify_kfd": False, "init_retry_s": 0.0}
        cfg.update(over)
        ex = core.Exporter(cfg)
        err = ex.start()
        made.append(ex)
        return ex, err

    yield make
    for ex in made:
        ex.stop()


def test_enumeration_sorted_by_hip_id_and_statics(fake_exporter):
    ex, err = fake_exporter({"FAKE_AMDSMI_GPUS": 4})
    assert err == ""
    st = ex.statics()
    assert [s["gpu_id"] for s in st] == ["0", "1", "2", "3"]  # the fake hands them out reversed
    assert st[1]["bdf"] == "0000:46:00.0"
    assert st[0]["gfx_target"] == "gfx950" and st[0]["num_cu"] == 256
    assert st[0]["power_limit_w"] == 1400  # microwatt power_limit normalised
    assert st[0]["compute_partition"] == "SPX" and st[0]["memory_partition"] == "NPS1"
    assert st[0]["vram_total_bytes"] == 294896 * 2 ** 20


def test_metrics_table_fields_and_na_omission(fake_exporter):
    ex, _ = fake_exporter()
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "node_gpu_gpu_util", gpu_id="0") == 37
    assert promtext.one(fam, "node_gpu_mem_bw_util", gpu_id="0") == 12
    assert not promtext.values(fam, "gpu_temperature_celsius", gpu_id="0", sensor="edge")  # N/A
    assert promtext.one(fam, "gpu_temperature_celsius", gpu_id="1", sensor="hotspot") == 47
    assert promtext.one(fam, "gpu_pcie_link_speed_gts", gpu_id="0") == 32
    assert len(promtext.values(fam, "gpu_xcd_busy_percent", gpu_id="0")) == 8
    clk = promtext.values(fam, "gpu_xcd_clock_mhz", gpu_id="0")
    assert sorted(clk) == [2093, 2094, 2095, 2096, 2097, 2098, 2099, 2100]
    links = {l["link"]: (l["peer_bdf"], v) for _, l, v in fam["gpu_xgmi_link_up"]["samples"] if l["gpu_id"] == "0"}
    assert set(links) == {str(k) for k in range(1, 8)}  # slot 0 (N/A status) is not a link
    assert links["3"] == ("0000:43:00.0", 1)
    assert promtext.one(fam, "gpu_xgmi_link_max_bandwidth_bytes_per_second", gpu_id="0", link="1") == 76e9
    assert "gpu_fan_rpm" not in fam and "gpu_voltage_volts" not in fam  # all N/A


def test_rates_from_accumulators(fake_exporter):
    ex, _ = fake_exporter()
    ex.tick()
    r = ex.rates()[0]
    assert r["valid"] and r["dt_s"] == pytest.approx(1.0)  # driver timestamp, not host time
    assert r["power_from_energy_w"] == pytest.approx(15.3, rel=1e-3)
    assert r["gfx_activity_avg_pct"] == pytest.approx(37.0)
    assert r["ppt_violation_pct"] == pytest.approx(10.0)
    assert r["xcd_busy_avg"] == pytest.approx([37.0] * 8)
    assert r["xgmi_rd_Bps"][3] == pytest.approx(3 * 1024e6)
    fam = promtext.parse(ex.metrics_text())
    u = promtext.one(fam, "gpu_xgmi_link_utilization_ratio", gpu_id="0", link="7")
    assert u == pytest.approx((7 * 1024e6 + 3.5 * 1024e6) * 8 / (608e9 * 2))


def test_process_list_resize_path(fake_exporter):
    ex, _ = fake_exporter({"FAKE_AMDSMI_GPUS": 1, "FAKE_AMDSMI_PROCS": 150})
    ex.tick()
    rows = ex.pod_rows()
    assert len(rows) == 150  # > the initial 64-entry buffer: OUT_OF_RESOURCES -> grow -> retry
    assert {r["procname"] for r in rows} >= {"worker-0", "worker-149"}
    assert max(r["used_memory_bytes"] for r in rows) == 150 * 2 ** 30


def test_per_device_failure_isolated(fake_exporter):
    ex, _ = fake_exporter({"FAKE_AMDSMI_GPUS": 3, "FAKE_AMDSMI_FAIL_METRICS": 1})
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    # gpu 1 lost its metrics table but VRAM still answers -> still "up" with partial data
    assert promtext.one(fam, "gpu_up", gpu_id="1") == 1
    assert not promtext.values(fam, "node_gpu_gpu_util", gpu_id="1")
    assert promtext.one(fam, "node_gpu_mem_used", gpu_id="1") == 283 + 1024
    assert promtext.one(fam, "gpumon_sample_errors_total", gpu_id="1") >= 1
    assert promtext.one(fam, "gpumon_backend_call_errors_total", call="gpu_metrics") >= 1
    assert promtext.one(fam, "node_gpu_gpu_util", gpu_id="2") == 37


def test_no_metrics_table_falls_back_to_activity_api(fake_exporter):
    ex, _ = fake_exporter({"FAKE_AMDSMI_GPUS": 2, "FAKE_AMDSMI_NO_METRICS": 1})
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "node_gpu_gpu_util", gpu_id="1") == 12  # amdsmi_get_gpu_activity
    assert promtext.one(fam, "gpumon_backend_calls_total", call="gpu_activity") >= 2


def _calls(fam, call):
    return promtext.one(fam, "gpumon_backend_calls_total", call=call)


def test_unsupported_queries_latch_off_per_device_and_field(fake_exporter):
    """A query the firmware / partition mode does not offer (NOT_SUPPORTED) is dropped for good
    after its first answer, per call: the fields it fed are omitted, the rest keep flowing, and no
    error is counted. Without any query that answers the GPU is down."""
    ex, _ = fake_exporter({"FAKE_AMDSMI_NO_METRICS": 1, "FAKE_AMDSMI_UNSUPPORTED": "activity,power"})
    for _ in range(3):
        ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert "node_gpu_gpu_util" not in fam and "gpu_power_watts" not in fam
    assert promtext.one(fam, "node_gpu_mem_used", gpu_id="1") == 1307
    assert promtext.values(fam, "gpu_up") == [1, 1]
    assert _calls(fam, "gpu_activity") == 2 and _calls(fam, "power_info") == 2  # once per GPU, then latched
    assert _calls(fam, "vram_usage") == 8  # start() + 3 ticks, 2 GPUs
    assert promtext.values(fam, "gpumon_sample_errors_total") == [0, 0]

    ex, _ = fake_exporter({"FAKE_AMDSMI_NO_METRICS": 1, "FAKE_AMDSMI_UNSUPPORTED": "activity,power,vram"})
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.values(fam, "gpu_up") == [0, 0]
    assert "node_gpu_mem_used" not in fam


def test_transient_errors_are_counted_and_retried(fake_exporter):
    ex, _ = fake_exporter({"FAKE_AMDSMI_NO_METRICS": 1, "FAKE_AMDSMI_BUSY": "vram"})
    ex.tick()
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.values(fam, "gpu_up") == [1, 1]  # activity still answers
    assert promtext.one(fam, "node_gpu_gpu_util", gpu_id="1") == 12
    assert "node_gpu_mem_used" not in fam
    assert promtext.values(fam, "gpumon_sample_errors_total") == [3, 3]  # every tick, never latched
    assert _calls(fam, "vram_usage") == 6


def test_process_list_support_and_failures(fake_exporter):
    """A device whose library cannot list processes is not failing: no failures counted, no held
    list. A list that fails (BUSY) on a device that can is counted; having never listed, it holds
    nothing."""
    ex, _ = fake_exporter({"FAKE_AMDSMI_UNSUPPORTED": "procs"})
    ex.tick()
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.values(fam, "gpu_process_count") == [0, 0]
    assert promtext.one(fam, "gpumon_process_list_failures_total") == 0
    assert "gpu_process_list_held" not in fam
    assert _calls(fam, "process_list") == 2  # latched after the first answer
    ex, _ = fake_exporter({"FAKE_AMDSMI_BUSY": "procs"})
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpumon_process_list_failures_total") == 4  # start() + 1 tick, 2 GPUs
    assert promtext.values(fam, "gpu_process_list_held") == [0, 0]


def test_link_metrics_unsupported_or_failing(fake_exporter):
    ex, _ = fake_exporter({"FAKE_AMDSMI_UNSUPPORTED": "links"})
    for _ in range(3):
        ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert _calls(fam, "link_metrics") == 2  # asked once per GPU, then latched
    assert promtext.values(fam, "gpu_xgmi_read_bytes_per_second", gpu_id="0")  # the table's traffic stays
    ex, _ = fake_exporter({"FAKE_AMDSMI_BUSY": "links"})
    for _ in range(3):
        ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert _calls(fam, "link_metrics") == 8  # a failed refresh is retried on the next tick


def test_init_failure_then_recovery(fake_exporter, monkeypatch):
    ex, err = fake_exporter({"FAKE_AMDSMI_INIT_FAIL": 1})
    assert "INIT_ERROR" in err
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpumon_backend_up") == 0
    monkeypatch.delenv("FAKE_AMDSMI_INIT_FAIL")
    ex.tick()  # init_retry_s = 0: retried on the next tick
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpumon_backend_up") == 1
    assert len(promtext.values(fam, "node_gpu_gpu_util")) == 2


def test_device_filter_and_replicate(fake_exporter):
    ex, _ = fake_exporter({"FAKE_AMDSMI_GPUS": 4}, devices=[2], backend="amdsmi:replicate=3")
    st = ex.statics()
    assert [s["gpu_id"] for s in st] == ["2", "1", "2"] or len(st) == 3
    assert all(s["bdf"] == "0000:66:00.0" for s in st)


def test_cpx_partition_mode(fake_exporter):
    """CPX: 8 logical GPUs per socket, each with ONE XCD whose counters live in
    xcp_stats[partition_id] (SURVEY.md §7.3 hard part 2)."""
    ex, err = fake_exporter({"FAKE_AMDSMI_GPUS": 2, "FAKE_AMDSMI_CPX": 1})
    assert err == ""
    st = ex.statics()
    assert len(st) == 16
    assert [s["gpu_id"] for s in st] == [str(i) for i in range(16)]
    assert {s["compute_partition"] for s in st} == {"CPX"}
    assert [s["partition_id"] for s in st[:8]] == list(range(8))
    assert st[3]["bdf"] == "0000:26:00.3" and st[11]["bdf"] == "0000:46:00.3"
    ex.tick()
    ex.tick()
    for i in (0, 3, 9):
        sm = ex.samples()[i]
        assert sm["xcd_busy"] == [10 * (i % 8) + 5]  # exactly one XCD, from its own XCP slot
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpu_xcd_busy_percent", gpu_id="3", xcd="0") == 35
    assert promtext.one(fam, "gpu_xcd_busy_avg_percent", gpu_id="3", xcd="0") == pytest.approx(35)
    assert len(promtext.values(fam, "gpu_xcd_busy_percent")) == 16


# The string libamd_smi returned on the pool's MI355X boxes (amdgpu in the kernel: /proc/version
# with its spaces removed), which the exporter used to cut to 64 bytes into the gpu_info label
# (profiles/data/r4/cm_base.prom:24).
POOL_DRIVER_STRING = "Linuxversion6.18.51-ant.1(nixbld@localhost)(gcc(GCC)15.3.0,GNUld(GNUBinutils)2.46)#1-ant-ociSMP"


def test_driver_version_label_from_proc_version_string(fake_exporter, tmp_path):
    ex, err = fake_exporter({"FAKE_AMDSMI_DRIVER_VERSION": POOL_DRIVER_STRING}, sysfs_root=str(tmp_path))
    assert err == ""
    st = ex.statics()[0]
    assert st["driver_version"] == "6.18.51-ant.1" and st["driver_source"] == "kernel"
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    (_, lab, _), *_ = fam["gpu_info"]["samples"]
    assert lab["driver_version"] == "6.18.51-ant.1" and lab["driver_source"] == "kernel"


def test_driver_version_label_prefers_the_module_version(fake_exporter, tmp_path):
    (tmp_path / "module" / "amdgpu").mkdir(parents=True)
    (tmp_path / "module" / "amdgpu" / "version").write_text("6.12.12\n")
    ex, err = fake_exporter({"FAKE_AMDSMI_DRIVER_VERSION": POOL_DRIVER_STRING}, sysfs_root=str(tmp_path))
    assert err == ""
    st = ex.statics()[0]
    assert st["driver_version"] == "6.12.12" and st["driver_source"] == "module"


@pytest.mark.parametrize("raw,want", [
    ("Linux version 6.8.0-45-generic (buildd@lcy02-amd64-075) (x86_64-linux-gnu-gcc-13 (Ubuntu 13.2.0)",
     ("6.8.0-45-generic", "kernel")),
    (POOL_DRIVER_STRING, ("6.18.51-ant.1", "kernel")),
    ("6.10.5", ("6.10.5", "library")),
    # a long library string is cut at a separator, never inside a token
    ("amdgpu 6.10.5 " + "x" * 40 + " build 1234567890 extra-tail-token", ("amdgpu 6.10.5 " + "x" * 40 + " build", "library")),
])
def test_driver_version_label_rules(core, raw, want):
    got = core.driver_version_label(raw, "")
    assert tuple(got) == want and len(got[0]) <= 64 and " " not in got[0].strip().split(" ")[-1]


def test_driver_version_label_empty_falls_back_to_the_kernel_release(core):
    v, src = core.driver_version_label("", "")
    assert src == "kernel" and v == os.uname().release


def test_pcie_interval_rate_from_the_accumulator(fake_exporter):
    """gpu_pcie_bandwidth_bytes_per_second is d(pcie_bandwidth_acc) over the
    firmware's accumulation ticks x pcie_bw_unit_bytes (102400 B/s per unit, measured on MI355X);
    the instantaneous gauge is the same unit; the old GB/s-labelled family is gone."""
    ex, err = fake_exporter({"FAKE_AMDSMI_GPUS": 2})
    assert err == ""
    ex.tick()
    ex.tick()
    r = ex.rates()
    # the fake adds (500000 + 1000 d) units per accumulation tick
    assert r[0]["pcie_Bps"] == pytest.approx(500000 * 102400.0)
    assert r[1]["pcie_Bps"] == pytest.approx(501000 * 102400.0)
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpu_pcie_bandwidth_bytes_per_second", gpu_id="0") == pytest.approx(51.2e9)
    assert promtext.one(fam, "gpu_pcie_bandwidth_inst_bytes_per_second", gpu_id="0") == 18 * 102400.0
    assert "gpu_pcie_bandwidth_gbytes_per_second" not in fam


def test_pcie_unit_is_configurable(fake_exporter):
    ex, err = fake_exporter(pcie_bw_unit_bytes=1000.0)
    assert err == ""
    ex.tick()
    ex.tick()
    assert ex.rates()[0]["pcie_Bps"] == pytest.approx(500000 * 1000.0)
