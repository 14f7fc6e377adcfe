"""The REAL RocmSmiBackend (rocm_smi_lib fallback) exercised on CPU against
build/fakes/libfake_rocm_smi.so (csrc/fakes/fake_rocm_smi.cpp): same MI355X gpu_metrics table as
the amdsmi fake, so the exposition must match field for field; plus the `auto` fallback from a
failing libamd_smi to rocm_smi."""

import os

import pytest

from conftest import make_locked
from gpumon.export import promtext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE_RSMI = os.path.join(ROOT, "build", "fakes", "libfake_rocm_smi.so")
FAKE_AMDSMI = os.path.join(ROOT, "build", "fakes", "libfake_amd_smi.so")
ENV_KEYS = ("FAKE_RSMI_GPUS", "FAKE_RSMI_PROCS", "FAKE_RSMI_FAIL_METRICS", "FAKE_RSMI_INIT_FAIL",
            "FAKE_RSMI_NO_METRICS", "FAKE_AMDSMI_GPUS", "FAKE_AMDSMI_INIT_FAIL", "FAKE_AMDSMI_PROCS",
            "FAKE_AMDSMI_FAIL_METRICS", "FAKE_AMDSMI_NO_METRICS")


@pytest.fixture(scope="module", autouse=True)
def fake_libs():
    make_locked("fakes")


@pytest.fixture
def make_exporter(core, monkeypatch):
    made = []

    def make(env=None, **over):
        for k in ENV_KEYS:
            monkeypatch.delenv(k, raising=False)
        for k, v in (env or {}).items():
            monkeypatch.setenv(k, str(v))
        cfg = {"backend": "rocm_smi", "rocm_smi_lib": FAKE_RSMI, "serve_http": False, "interval_s": 0,
               "host": "n1", "verify_kfd": False, "init_retry_s": 0.0}
        cfg.update(over)
        ex = core.Exporter(cfg)
        err = ex.start()
        made.append(ex)
        return ex, err

    yield make
    for ex in made:
        ex.stop()


def test_statics(make_exporter):
    ex, err = make_exporter({"FAKE_RSMI_GPUS": 3})
    assert err == ""
    st = ex.statics()
    assert [s["gpu_id"] for s in st] == ["0", "1", "2"]
    assert st[1]["bdf"] == "0000:46:00.0"  # rsmi BDFID decoded
    assert st[0]["power_limit_w"] == 1400
    assert st[0]["vram_total_bytes"] == 288 * 2 ** 30
    assert st[0]["compute_partition"] == "SPX"
    assert "fake rocm_smi" in st[0]["model"]
    assert ex.self_stats()["backend"] == "rocm_smi"
    assert ex.self_stats()["backend_version"] == "77.1.2"


def test_same_firmware_table_as_amdsmi(make_exporter):
    """Both backends decode the same gpu_metrics table through metrics_table.h: the per-device
    firmware families must be identical."""
    rs, _ = make_exporter()
    am, err = make_exporter(backend="amdsmi", amdsmi_lib=FAKE_AMDSMI)
    assert err == ""
    for ex in (rs, am):
        ex.tick()
        ex.tick()
    fr, fa = promtext.parse(rs.metrics_text()), promtext.parse(am.metrics_text())
    for name in ("gpu_temperature_celsius", "gpu_power_watts", "gpu_xcd_busy_percent", "gpu_clock_mhz",
                 "gpu_gfx_activity_avg_percent", "gpu_xgmi_read_bytes_per_second", "gpu_violation_percent",
                 "gpu_pcie_link_width", "node_gpu_gpu_util"):
        assert name in fr, name
        assert sorted(promtext.values(fr, name)) == pytest.approx(sorted(promtext.values(fa, name))), name
    # energy-derived power: 1e6 counts x 15.3 uJ per simulated second
    assert rs.rates()[0]["power_from_energy_w"] == pytest.approx(15.3, rel=1e-3)


def test_processes_and_resize(make_exporter):
    ex, _ = make_exporter({"FAKE_RSMI_GPUS": 2, "FAKE_RSMI_PROCS": 40})  # 80 node-wide > 64 first buffer
    ex.tick()
    rows = ex.pod_rows()
    pids = {(r["dev"], r["pid"]) for r in rows}
    assert len(pids) == 80
    assert {int(p) for g, p in pids if g == 1} == set(range(201000, 201040))
    assert {r["cu_occupancy"] for r in rows} == {64}
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpu_process_count", gpu_id="0") == 40


def test_busy_percent_fallback(make_exporter):
    ex, _ = make_exporter({"FAKE_RSMI_NO_METRICS": 1, "FAKE_RSMI_GPUS": 2})
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "node_gpu_gpu_util", gpu_id="1") == 12
    assert promtext.one(fam, "node_gpu_mem_used", gpu_id="1") == pytest.approx(283 + 1024)


def test_one_failing_device(make_exporter):
    ex, _ = make_exporter({"FAKE_RSMI_FAIL_METRICS": 1, "FAKE_RSMI_GPUS": 3})
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpu_up", gpu_id="1") == 1  # VRAM still answers
    assert promtext.one(fam, "gpumon_sample_errors_total", gpu_id="1") >= 1
    assert "gpu_id=\"1\"" not in "".join(l for l in ex.metrics_text().splitlines()
                                          if l.startswith("gpu_xcd_busy_percent"))


def test_init_failure_is_reported(make_exporter):
    ex, err = make_exporter({"FAKE_RSMI_INIT_FAIL": 1})
    assert "rsmi_init failed" in err
    assert promtext.one(promtext.parse(ex.metrics_text()), "gpumon_backend_up") == 0


def test_auto_falls_back_to_rocm_smi(make_exporter):
    ex, err = make_exporter({"FAKE_AMDSMI_INIT_FAIL": 1, "FAKE_RSMI_GPUS": 2}, backend="auto",
                            amdsmi_lib=FAKE_AMDSMI)
    assert err == ""
    assert ex.self_stats()["backend"] == "rocm_smi"
    ex.tick()
    assert promtext.values(promtext.parse(ex.metrics_text()), "gpu_up") == [1, 1]


def test_auto_prefers_amdsmi(make_exporter):
    ex, err = make_exporter({"FAKE_AMDSMI_GPUS": 1}, backend="auto", amdsmi_lib=FAKE_AMDSMI)
    assert err == ""
    assert ex.self_stats()["backend"] == "amdsmi"
