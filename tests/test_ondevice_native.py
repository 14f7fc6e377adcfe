"""Native on-device samplers (csrc/core/ondevice.cpp) on CPU, through the same dlopen path the
exporter uses on a GPU node, against the fake plugins of csrc/fakes/fake_ondevice.cpp.

The real plugins (lib/libgpumon_pmc.so, lib/libgpumon_probe.so) are covered on the MI355X by
tests/test_gpu_pmc.py and tests/test_gpu_cli.py."""

import os
import re
import subprocess

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from conftest import ROOT, make_locked
from oracles.ops.pmc import derive

FAKE_DIR = os.path.join(ROOT, "build", "fakes", "ondevice")
BIN = os.path.join(ROOT, "bin", "gpumon-exporter")


@pytest.fixture(scope="module", autouse=True)
def fakes():
    make_locked("fakes")
    make_locked("core")


def _val(text, name, **labels):
    for line in text.splitlines():
        if not line.startswith(name + "{"):
            continue
        if all(f'{k}="{v}"' in line for k, v in labels.items()):
            return float(line.rsplit(" ", 1)[1])
    return None


def _ondevice(core, ex, **over):
    cfg = {"plugin_dir": FAKE_DIR, "pmc": True, "probe": True, "pmc_every_s": 0.2, "probe_every_s": 0.2,
           "pmc_window_s": 0.01, "pmc_mode": "window"}
    cfg.update(over)
    return core.OnDevice(ex, cfg)


# ---------------------------------------------------------------- derivation parity (C++ vs Python)
AGENT = {"cu_count": 256, "simd_count": 1024, "max_waves_per_cu": 32, "num_xcc": 8}
_pos = st.floats(min_value=0, max_value=1e12, allow_nan=False)


@settings(max_examples=200, deadline=None)
@given(gui=_pos, cnt=_pos, mfma=_pos, waves=_pos, nx=st.integers(0, 8), has=st.lists(st.booleans(), min_size=5,
                                                                                     max_size=5),
       mops=_pos, window=st.sampled_from([0.0, 0.05, 0.1]))
def test_pmc_derive_matches_python(gui, cnt, mfma, waves, nx, has, mops, window):
    raw = {}
    if has[0]:
        raw["GRBM_GUI_ACTIVE"] = {"sum": gui * 8, "max": gui, "n": 8, "by_xcc": []}
    if has[1]:
        raw["GRBM_COUNT"] = {"sum": cnt * 8, "max": cnt, "n": 8, "by_xcc": []}
    if has[2]:
        raw["SQ_VALU_MFMA_BUSY_CYCLES"] = {"sum": mfma, "max": mfma, "n": 8, "by_xcc": [mfma / nx] * nx if nx else []}
    if has[3]:
        raw["SQ_WAVE_CYCLES"] = {"sum": waves, "max": waves, "n": 8, "by_xcc": []}
    if has[4]:
        raw["SQ_INSTS_VALU_MFMA_MOPS_BF16"] = {"sum": mops, "max": mops, "n": 8, "by_xcc": []}
        raw["SQ_INSTS_VALU_MFMA_MOPS_F6F4"] = {"sum": mops / 3, "max": mops, "n": 8, "by_xcc": []}
    from gpumon import core

    py = derive(raw, AGENT, window)
    cc = core().pmc_derive(raw, AGENT, window)
    assert set(py) == set(cc)
    for k in py:
        assert cc[k] == pytest.approx(py[k], rel=1e-12)


def test_default_plugin_dir_is_tree_lib(core, monkeypatch):
    monkeypatch.delenv("GPUMON_PLUGIN_DIR", raising=False)
    assert os.path.realpath(core.default_plugin_dir()) == os.path.join(os.path.realpath(ROOT), "lib")
    monkeypatch.setenv("GPUMON_PLUGIN_DIR", "/elsewhere")
    assert core.default_plugin_dir() == "/elsewhere"


# ---------------------------------------------------------------- in-process (gpumon._core.OnDevice)
def test_native_samplers_export_series(core, mock_exporter, monkeypatch):
    monkeypatch.setenv("GPUMON_FAKE_AGENTS", "2")
    monkeypatch.setenv("GPUMON_FAKE_MFMA", "0.75")
    monkeypatch.setenv("GPUMON_FAKE_OCC", "0.5")
    monkeypatch.setenv("GPUMON_FAKE_TFLOPS", "2000")
    ex = mock_exporter()
    od = _ondevice(core, ex)
    od.start()
    try:
        assert od.step()
        ex.tick()
        m = ex.metrics_text()
        for g in ("0", "1"):
            assert _val(m, "gpu_mfma_busy_active_percent", gpu_id=g) == pytest.approx(75.0)
            assert 0 < _val(m, "gpu_mfma_util_percent", gpu_id=g) <= 75.0  # x wall-time activity
            assert _val(m, "gpu_pmc_coverage_ratio", gpu_id=g) == pytest.approx(0.01 / 0.2)
            assert _val(m, "gpu_mfma_tflops", gpu_id=g, dtype="bf16") == pytest.approx(2000.0)
            assert _val(m, "gpu_mfma_tflops", gpu_id=g, dtype="f16") == pytest.approx(200.0)
            assert _val(m, "gpu_mfma_tflops", gpu_id=g, dtype="f64") == 0
            assert _val(m, "gpu_occupancy_percent", gpu_id=g) is None  # no wave counters by default
            assert _val(m, "gpu_gui_active_percent", gpu_id=g) == pytest.approx(100.0)
            assert _val(m, "gpu_pmc_window_seconds", gpu_id=g) == pytest.approx(0.01)
            for x in range(8):
                assert _val(m, "gpu_xcd_mfma_busy_active_percent", gpu_id=g, xcd=x) == pytest.approx(75.0)
                assert _val(m, "gpu_probe_xcd_blocks", gpu_id=g, xcd=x) == 1024 / 8
                assert _val(m, "gpu_probe_xcd_clock_mhz", gpu_id=g, xcd=x) == pytest.approx(2400 - 10 * x)
            assert _val(m, "gpu_probe_unique_cus", gpu_id=g) == 256
            assert _val(m, "gpu_probe_wave_slot_mean", gpu_id=g) == pytest.approx(1.75)
            assert _val(m, "gpu_probe_xcd_wave_slot_mean", gpu_id=g, xcd=6) == pytest.approx(3.0)
            assert _val(m, "gpu_probe_pending", gpu_id=g) == 0
        assert "# TYPE gpumon_pmc_errors_total counter" in m
        s = od.stats()
        assert s["pmc_agents"] == 2 and s["probe_devices"] == 2 and s["pmc_samples"] >= 2 and s["probe_done"] >= 2
    finally:
        od.stop()
    ex.tick()
    m = ex.metrics_text()
    assert "gpu_mfma_util_percent" not in m and "gpu_probe_pending" not in m  # series withdrawn on stop


def test_explicit_wave_counter_gives_occupancy(core, mock_exporter, monkeypatch):
    monkeypatch.setenv("GPUMON_FAKE_OCC", "0.5")
    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, probe=False, pmc_counters=["SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE", "GRBM_COUNT"])
    od.start()
    try:
        od.step()
        ex.tick()
        m = ex.metrics_text()
        assert _val(m, "gpu_occupancy_percent", gpu_id="0") == pytest.approx(50.0)
        assert "gpu_mfma_tflops" not in m
    finally:
        od.stop()


def test_background_threads_keep_sampling(core, mock_exporter, monkeypatch):
    import time

    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, pmc_every_s=0.05, probe_every_s=0.05)
    od.start()
    try:
        t0 = time.monotonic()
        while time.monotonic() - t0 < 5 and (od.stats()["pmc_samples"] < 5 or od.stats()["probe_done"] < 5):
            time.sleep(0.02)
        s = od.stats()
        assert s["pmc_samples"] >= 5 and s["probe_done"] >= 5 and s["pmc_errors"] == 0
    finally:
        t0 = time.monotonic()
        od.stop()
        assert time.monotonic() - t0 < 2  # the waits are interruptible


def test_pmc_init_failure_fails_loudly(core, mock_exporter, monkeypatch):
    monkeypatch.setenv("GPUMON_FAKE_PMC_FAIL", "init")
    od = _ondevice(core, mock_exporter())
    with pytest.raises(RuntimeError, match="device counting unavailable"):
        od.start()


def test_missing_plugin_fails_loudly(core, mock_exporter, tmp_path):
    od = _ondevice(core, mock_exporter(), plugin_dir=str(tmp_path), ondevice_isolate=False)
    with pytest.raises(RuntimeError, match="dlopen .*libgpumon_pmc.so"):
        od.start()


def test_sample_failures_counted(core, mock_exporter, monkeypatch):
    monkeypatch.setenv("GPUMON_FAKE_PMC_FAIL", "sample")
    ex = mock_exporter()
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, ondevice_isolate=False)
    od.start()
    try:
        od.step()
        ex.tick()
        m = ex.metrics_text()
        assert "gpu_mfma_util_percent" not in m
        assert re.search(r'^gpumon_pmc_errors_total\{host="node-a"\} [1-9]', m, re.M)  # node-level series
        assert od.stats()["pmc_errors"] >= 1
    finally:
        od.stop()


def test_probe_timeouts(core, mock_exporter, monkeypatch):
    monkeypatch.setenv("GPUMON_FAKE_PROBE_HANG", "1")
    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, pmc=False, probe_every_s=60, probe_timeout_s=0.01)
    od.start()
    try:
        od.step()
        od.step()
        ex.tick()
        m = ex.metrics_text()
        assert _val(m, "gpu_probe_timeouts_total", gpu_id="0") >= 2  # + the background thread's first step
        assert _val(m, "gpu_probe_pending", gpu_id="0") == 1
        assert "gpu_probe_latency_seconds" not in m
    finally:
        monkeypatch.delenv("GPUMON_FAKE_PROBE_HANG")
        od.stop()


# ---------------------------------------------------------------- standalone binary + Python CLI
def _run_bin(*args, env=None):
    e = dict(os.environ, GPUMON_FAKE_AGENTS="2")
    e.update(env or {})
    return subprocess.run([BIN, "--backend", "mock:gpus=2", "--once", "--no-pod-resources", "--no-cri", *args],
                          capture_output=True, text=True, timeout=60, env=e)


def test_binary_pmc_and_probe_flags():
    r = _run_bin("--pmc", "--probe", "--plugin-dir", FAKE_DIR, env={"GPUMON_FAKE_MFMA": "0.25"})
    assert r.returncode == 0, r.stderr
    assert _val(r.stdout, "gpu_mfma_busy_active_percent", gpu_id="1") == pytest.approx(25.0)
    assert _val(r.stdout, "gpu_pmc_coverage_ratio", gpu_id="1") == 1  # continuous by default
    assert _val(r.stdout, "gpu_probe_xcd_blocks", gpu_id="1", xcd="7") == 128


def test_binary_plugin_dir_from_env():
    r = _run_bin("--probe", env={"GPUMON_PLUGIN_DIR": FAKE_DIR})
    assert r.returncode == 0, r.stderr
    assert "gpu_probe_unique_cus" in r.stdout and "gpu_mfma_util_percent" not in r.stdout


def test_binary_missing_plugin_exits_nonzero(tmp_path):
    r = _run_bin("--pmc", "--plugin-dir", str(tmp_path))
    assert r.returncode == 1 and "gpumon-ondevice-helper" in r.stderr


def test_binary_without_flags_loads_no_plugin():
    r = _run_bin(env={"GPUMON_PLUGIN_DIR": "/nonexistent"})
    assert r.returncode == 0 and "gpu_probe" not in r.stdout


def test_cli_once_native_ondevice(monkeypatch, capsys):
    from gpumon import cli

    monkeypatch.setenv("GPUMON_FAKE_AGENTS", "1")
    rc = cli.main(["once", "--backend", "mock:gpus=1", "--enable-pmc", "--enable-probe-kernel",
                   "--plugin-dir", FAKE_DIR, "--control-plane", "off"])
    out = capsys.readouterr().out
    assert rc == 0
    assert _val(out, "gpu_mfma_busy_active_percent", gpu_id="0") == pytest.approx(50.0)
    assert _val(out, "gpu_probe_unique_cus", gpu_id="0") == 256


def test_probe_created_once_backend_comes_up(core, monkeypatch):
    """Backend down at start (no device list yet): the probe sampler starts with nothing to probe and
    creates its probes on the first step after the exporter's backend initialises."""
    make_locked("fakes")
    fake = os.path.join(ROOT, "build", "fakes", "libfake_amd_smi.so")
    monkeypatch.setenv("GPUMON_FAKE_AGENTS", "2")
    monkeypatch.setenv("FAKE_AMDSMI_INIT_FAIL", "1")
    ex = core.Exporter({"backend": "amdsmi", "amdsmi_lib": fake, "serve_http": False, "interval_s": 0,
                        "init_retry_s": 0.0, "verify_kfd": False, "sysfs_root": "/nonexistent"})
    assert ex.start() != ""  # backend not ready yet (retrying)
    od = _ondevice(core, ex, pmc=False, probe_every_s=60)
    od.start()
    try:
        od.step()
        assert od.stats()["probe_devices"] == 0
        monkeypatch.delenv("FAKE_AMDSMI_INIT_FAIL")
        ex.tick()
        assert len(ex.statics()) == 2
        od.step()
        ex.tick()
        assert od.stats()["probe_devices"] == 2
        assert _val(ex.metrics_text(), "gpu_probe_unique_cus", gpu_id="1") == 256
    finally:
        od.stop()
        ex.stop()


# ---------------------------------------------------------------- continuous counting
def test_continuous_counting_covers_every_interval(core, mock_exporter, monkeypatch):
    """Contexts stay started; each step reads the cumulative counts and exports the difference
    since the previous read: the counted span is the whole interval (coverage 1)."""
    import time

    monkeypatch.setenv("GPUMON_FAKE_MFMA", "0.6")
    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, pmc_mode="continuous")
    od.start()
    try:
        od.step()  # starts the contexts and reads again after one window
        time.sleep(0.15)
        od.step()
        ex.tick()
        m = ex.metrics_text()
        assert _val(m, "gpu_mfma_busy_active_percent", gpu_id="0") == pytest.approx(60.0)
        assert _val(m, "gpu_pmc_coverage_ratio", gpu_id="0") == 1
        assert 0.14 <= _val(m, "gpu_pmc_window_seconds", gpu_id="0") <= 0.5  # the whole gap between reads
        assert _val(m, "gpu_mfma_tflops", gpu_id="0", dtype="bf16") == pytest.approx(1000.0, rel=0.05)
        assert _val(m, "gpumon_pmc_up") == 1
        assert od.stats()["pmc_continuous"] and od.stats()["pmc_errors"] == 0
    finally:
        od.stop()


def test_continuous_counters_held_elsewhere(core, mock_exporter, monkeypatch):
    """Another profiler holds the device counters: no values (never stale ones), pmc_up 0, errors
    counted, and counting resumes once the counters are free again."""
    import time

    monkeypatch.setenv("GPUMON_FAKE_PMC_FAIL", "start")
    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, pmc_mode="continuous", ondevice_isolate=False)
    od.start()
    try:
        od.step()
        ex.tick()
        m = ex.metrics_text()
        assert _val(m, "gpumon_pmc_up") == 0 and "gpu_mfma_util_percent" not in m
        assert od.stats()["pmc_errors"] >= 1
        monkeypatch.delenv("GPUMON_FAKE_PMC_FAIL")
        od.step()
        time.sleep(0.05)
        od.step()
        ex.tick()
        m = ex.metrics_text()
        assert _val(m, "gpumon_pmc_up") == 1 and _val(m, "gpu_mfma_busy_active_percent", gpu_id="0") > 0
    finally:
        od.stop()


def test_continuous_restart_underneath_drops_the_interval(core, mock_exporter, monkeypatch):
    """Counts going backwards (contexts restarted by someone else) must not export a negative or
    garbage interval: it is dropped and counted in gpumon_pmc_resets_total."""
    import time

    monkeypatch.setenv("GPUMON_FAKE_PMC_RESTART", "3")
    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, pmc_mode="continuous")
    od.start()
    try:
        for _ in range(7):
            od.step()
            time.sleep(0.03)
            ex.tick()
            v = _val(ex.metrics_text(), "gpu_mfma_busy_active_percent", gpu_id="0")
            assert v is None or 0 <= v <= 100
        assert od.stats()["pmc_resets"] >= 1
        assert _val(ex.metrics_text(), "gpumon_pmc_resets_total") >= 1
    finally:
        od.stop()


# ---------------------------------------------------------------- helper process (ondevice_isolate)
def _helper_pids():
    out = []
    for p in os.listdir("/proc"):
        if p.isdigit():
            try:
                if open(f"/proc/{p}/comm").read().strip() == "gpumon-ondevice" and \
                        int(open(f"/proc/{p}/stat").read().rsplit(")", 1)[1].split()[1]) == os.getpid():
                    out.append(int(p))
            except (OSError, ValueError, IndexError):
                pass
    return out


def _state(pid, want=None, timeout=2.0):
    """The process state letter; with `want`, polls until it shows (SIGSTOP is delivered
    asynchronously, a loaded CPU may not have stopped the helper yet when kill() returns)."""
    import time

    deadline = time.time() + timeout
    while True:
        st = open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()[0]
        if want is None or st == want or time.time() > deadline:
            return st
        time.sleep(0.01)


def _kill(pid, timeout=5.0):
    """SIGKILL the helper and wait until it is dead (a zombie until the exporter reaps it): the
    signal is delivered asynchronously, and on a loaded CPU the next sampler step could otherwise
    still find it alive."""
    import signal
    import time

    os.kill(pid, signal.SIGKILL)
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            if open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()[0] in ("Z", "X"):
                return
        except OSError:
            return
        time.sleep(0.005)


def _after_first_loop_step(od, timeout=10.0):
    """The PMC and probe sampler threads step once right after start(): wait for them, so a test's
    own steps and kills are not raced by them (on a loaded host they may run much later)."""
    import time

    deadline = time.time() + timeout
    while time.time() < deadline:
        st = od.stats()
        pmc_done = st["pmc_steps"] >= 1 or not st["pmc_agents"]
        probe_done = st["probe_steps"] >= 1 or not st["probe_devices"]
        if pmc_done and probe_done:
            return
        time.sleep(0.005)


def test_isolated_pmc_runs_in_a_frozen_helper(core, mock_exporter, monkeypatch):
    """ondevice_isolate (default): the counting contexts live in a child process that is stopped
    (SIGSTOP, state T) between requests and answers correctly when resumed; stop() ends it."""
    import time

    monkeypatch.setenv("GPUMON_FAKE_MFMA", "0.4")
    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, pmc_mode="continuous")
    od.start()
    try:
        pids = _helper_pids()
        assert len(pids) == 1
        od.step()
        time.sleep(0.05)
        od.step()
        assert _state(pids[0], "T") == "T"  # frozen between reads
        ex.tick()
        m = ex.metrics_text()
        assert _val(m, "gpumon_ondevice_helper_resident_memory_bytes") > 1 << 20  # the pod's footprint
        assert _val(m, "gpumon_ondevice_helper_cpu_seconds_total") >= 0
        assert _val(m, "gpu_mfma_busy_active_percent", gpu_id="0") == pytest.approx(40.0)
        assert _val(m, "gpu_pmc_coverage_ratio", gpu_id="0") == 1
    finally:
        od.stop()
    time.sleep(0.1)
    assert _helper_pids() == []  # reaped


def test_isolated_pmc_window_mode_and_errors(core, mock_exporter, monkeypatch):
    monkeypatch.setenv("GPUMON_FAKE_PMC_FAIL", "sample")
    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, pmc_mode="window")
    od.start()
    try:
        od.step()
        assert od.stats()["pmc_errors"] >= 1
        ex.tick()
        assert "gpu_mfma_util_percent" not in ex.metrics_text()
    finally:
        od.stop()


def test_isolated_pmc_helper_death_is_survived(core, mock_exporter):
    """A helper that dies (OOM-killed, crashed) turns into PMC errors, never a hang or a crash of
    the exporter."""

    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, pmc_mode="continuous")
    od.start()
    try:
        _after_first_loop_step(od)
        od.step()
        (pid,) = _helper_pids()
        _kill(pid)
        od.step()
        assert od.stats()["pmc_errors"] >= 1
        ex.tick()
        assert _val(ex.metrics_text(), "gpumon_pmc_up") == 0
    finally:
        od.stop()


def test_isolated_pmc_missing_helper_fails_loudly(core, mock_exporter, tmp_path):
    import shutil

    shutil.copy(os.path.join(FAKE_DIR, "libgpumon_pmc.so"), tmp_path)
    od = _ondevice(core, mock_exporter(), probe=False, plugin_dir=str(tmp_path))
    with pytest.raises(RuntimeError, match="gpumon-ondevice-helper"):
        od.start()


def test_isolated_probe_runs_in_the_helper(core, mock_exporter, monkeypatch):
    """ondevice_isolate: the K1 probe is created, launched and waited on through the same helper
    process as the counting contexts, so this process never maps the probe library (and with it
    the HIP runtime); a killed helper turns into probe timeouts, not a hang."""
    import time

    monkeypatch.setenv("GPUMON_FAKE_AGENTS", "2")
    ex = mock_exporter(backend="mock:gpus=2")
    od = _ondevice(core, ex, probe_every_s=60, pmc_every_s=60, probe_timeout_s=0.5)
    od.start()
    try:
        assert len(_helper_pids()) == 1  # one helper for both samplers
        od.step()
        time.sleep(0.05)
        od.step()
        ex.tick()
        m = ex.metrics_text()
        for g in ("0", "1"):
            assert _val(m, "gpu_probe_latency_seconds", gpu_id=g) is not None
        (pid,) = _helper_pids()
        assert _state(pid, "T") == "T"
        _kill(pid)
        t0 = time.monotonic()
        od.step()
        assert time.monotonic() - t0 < 5
        ex.tick()
        assert _val(ex.metrics_text(), "gpumon_pmc_up") == 0
    finally:
        od.stop()


@pytest.mark.parametrize("isolate", [False, True], ids=["in_process", "helper"])
def test_probe_devices_paired_by_pci_address(core, mock_exporter, monkeypatch, isolate):
    """The probe's runtime numbers GPUs by HIP ordinal, which HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES
    renumber; the exporter's gpu_id is node-wide. With the runtime seeing node GPUs 3 and 1 (in that
    order) as ordinals 0 and 1, the probes land on gpu_id 3 and 1 -- paired by PCI address, in-process
    and through the helper -- and the GPUs the runtime cannot see get none (round 3 paired by
    hip_id: ordinal 0 -> gpu_id 0)."""
    monkeypatch.setenv("GPUMON_FAKE_AGENTS", "2")
    monkeypatch.setenv("GPUMON_FAKE_PCI", "0000:65:00.0,0000:25:00.0")  # mock GPUs 3 and 1
    ex = mock_exporter(backend="mock:gpus=4")
    od = _ondevice(core, ex, pmc=False, probe_every_s=60, ondevice_isolate=isolate)
    od.start()
    try:
        od.step()
        ex.tick()
        m = ex.metrics_text()
        s = od.stats()
        assert s["probe_devices"] == 2 and s["probe_by_bdf"] is True
        for g in ("1", "3"):
            assert _val(m, "gpu_probe_xcd_blocks", gpu_id=g, xcd=0) is not None, g
        for g in ("0", "2"):
            assert _val(m, "gpu_probe_xcd_blocks", gpu_id=g, xcd=0) is None, g
    finally:
        od.stop()


def test_isolated_exporter_maps_no_plugin():
    """The deployed shape: bin/gpumon-exporter with --pmc --probe maps neither plugin (nor, on a GPU
    node, the runtimes behind them); its one child, the helper, maps both."""
    import time

    e = dict(os.environ, GPUMON_FAKE_AGENTS="2")
    p = subprocess.Popen([BIN, "--backend", "mock:gpus=2", "--listen", "127.0.0.1:0", "--interval", "0.1",
                          "--no-pod-resources", "--no-cri", "--pmc", "--probe", "--plugin-dir", FAKE_DIR,
                          "--log-level", "error"], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=e, text=True)
    try:
        kids = []
        for _ in range(50):
            time.sleep(0.1)
            kids = [int(k) for t in os.listdir(f"/proc/{p.pid}/task")  # any thread may be the parent
                    for k in open(f"/proc/{p.pid}/task/{t}/children").read().split()]
            if kids:
                break
        assert p.poll() is None and len(kids) == 1
        time.sleep(0.5)
        maps = open(f"/proc/{p.pid}/maps").read()
        assert "libgpumon_probe.so" not in maps and "libgpumon_pmc.so" not in maps
        helper = open(f"/proc/{kids[0]}/maps").read()
        assert "libgpumon_probe.so" in helper and "libgpumon_pmc.so" in helper
    finally:
        p.terminate()
        p.wait(20)


def test_helper_outlives_the_thread_that_started_it(core, mock_exporter, monkeypatch):
    """PR_SET_PDEATHSIG follows the spawning THREAD: the helper is spawned from a process-lifetime
    thread, so starting the samplers from a short-lived thread does not kill it when that ends."""
    import threading
    import time

    monkeypatch.setenv("GPUMON_FAKE_MFMA", "0.3")
    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, pmc_mode="continuous")
    t = threading.Thread(target=od.start)
    t.start()
    t.join()
    try:
        time.sleep(0.2)
        assert len(_helper_pids()) == 1
        od.step()
        time.sleep(0.05)
        od.step()
        assert od.stats()["pmc_errors"] == 0
        ex.tick()
        assert _val(ex.metrics_text(), "gpu_mfma_busy_active_percent", gpu_id="0") == pytest.approx(30.0)
    finally:
        od.stop()


def test_dead_helper_is_respawned_and_samplers_recover(core, mock_exporter, monkeypatch):
    """A helper that dies (OOM-killed, crashed) is respawned by the next sampler step once
    helper_retry_s has passed: PMC is re-initialised first (rocprofiler before HSA), the probes are
    recreated, values come back and gpumon_ondevice_helper_restarts_total counts it."""
    import time

    monkeypatch.setenv("GPUMON_FAKE_MFMA", "0.5")
    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, pmc_every_s=60, probe_every_s=60, pmc_mode="continuous", helper_retry_s=0.2)
    od.start()
    try:
        _after_first_loop_step(od)
        od.step()
        (pid,) = _helper_pids()
        _kill(pid)
        od.step()  # the dead helper is noticed: errors, series withdrawn
        ex.tick()
        m = ex.metrics_text()
        assert _val(m, "gpumon_pmc_up") == 0
        time.sleep(0.3)
        od.step()  # respawn + PMC init; the first continuous read only starts the new contexts
        time.sleep(0.05)
        od.step()
        st = od.stats()
        assert st["helper_restarts"] == 1
        (pid2,) = _helper_pids()
        assert pid2 != pid
        ex.tick()
        m = ex.metrics_text()
        assert _val(m, "gpumon_pmc_up") == 1
        assert _val(m, "gpu_mfma_busy_active_percent", gpu_id="0") == pytest.approx(50.0)
        assert _val(m, "gpu_probe_latency_seconds", gpu_id="0") is not None
        assert _val(m, "gpumon_ondevice_helper_restarts_total") == 1
    finally:
        od.stop()
    time.sleep(0.1)
    assert _helper_pids() == []


def test_pmc_mfma_util_lands_on_the_exclusive_process_row(core, mock_exporter, monkeypatch):
    """The PMC sampler publishes each device's wall-time MFMA utilisation to the exporter; the one
    process with waves on that GPU gets it as pod_gpu_mfma_util_percent."""
    import time

    monkeypatch.setenv("GPUMON_FAKE_MFMA", "0.6")
    ex = mock_exporter(backend="mock:gpus=1,mode=load", sample_threads=0,
                       mock={"procs": [{"pid": 31, "device": 0, "name": "train", "kfd_only": True}]})
    ex.mock_set_occ_series(0, [180.0])
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, pmc_mode="continuous")
    od.start()
    try:
        od.step()
        time.sleep(0.05)
        od.step()
        ex.tick()
        time.sleep(0.05)
        ex.tick()
        m = ex.metrics_text()
        dev = _val(m, "gpu_mfma_util_percent", gpu_id="0")
        assert dev is not None and dev > 0
        assert _val(m, "pod_gpu_mfma_util_percent", pid="31") == pytest.approx(dev)
    finally:
        od.stop()
    ex.tick()
    assert _val(ex.metrics_text(), "pod_gpu_mfma_util_percent", pid="31") is None  # withdrawn with PMC


def test_helper_that_keeps_dying_backs_off(core, mock_exporter):
    """A helper killed again right after each respawn (e.g. OOM under a tight limit) is retried
    after helper_retry_s, then 2x, 4x ... that long, not in a tight loop."""
    import time

    ex = mock_exporter(backend="mock:gpus=1")
    od = _ondevice(core, ex, probe=False, pmc_every_s=60, pmc_mode="continuous", helper_retry_s=0.5)
    od.start()
    try:
        respawn_at = []
        t0 = time.monotonic()
        od.step()
        for _ in range(3):
            n = od.stats()["helper_restarts"]
            (pid,) = _helper_pids()
            _kill(pid)
            while od.stats()["helper_restarts"] == n:
                assert time.monotonic() - t0 < 10
                time.sleep(0.02)
                od.step()
            respawn_at.append(time.monotonic())
        gaps = [b - a for a, b in zip(respawn_at, respawn_at[1:])]
        # respawn 1 is immediate; the next ones wait 0.5 s x 2^streak after the previous attempt
        # started. A gap is that wait plus the difference of two spawn times, which a loaded host
        # stretches by ~0.1 s either way: 0.5 + jitter, then 1.0 + jitter
        assert 0.4 <= gaps[0] < 0.9 and gaps[1] >= 0.85 and gaps[1] > gaps[0], gaps
    finally:
        od.stop()


def test_silent_xcd_is_exported_as_zero_blocks(core, mock_exporter, monkeypatch):
    """K1 liveness: an XCD that ran none of the probe's workgroups reads 0 in gpu_probe_xcd_blocks
    (an alertable value), instead of its series disappearing."""
    monkeypatch.setenv("GPUMON_FAKE_DEAD_XCD", "3")
    ex = mock_exporter(backend="mock:gpus=1,n_xcd=8")
    ex.tick()
    od = _ondevice(core, ex, pmc=False, probe_every_s=60)
    od.start()
    try:
        od.step()
        ex.tick()
        m = ex.metrics_text()
        blocks = {x: _val(m, "gpu_probe_xcd_blocks", gpu_id="0", xcd=str(x)) for x in range(8)}
        assert blocks[3] == 0 and all(v > 0 for x, v in blocks.items() if x != 3), blocks
    finally:
        od.stop()


def test_helper_starts_with_a_clean_signal_mask():
    """The exporter binary blocks SIGTERM / SIGINT for its own handling; a signal mask survives
    exec, so the helper is spawned with an empty mask and default dispositions."""
    import time

    e = dict(os.environ, GPUMON_FAKE_AGENTS="1")
    p = subprocess.Popen([BIN, "--backend", "mock:gpus=1", "--listen", "127.0.0.1:0", "--interval", "0.2",
                          "--no-pod-resources", "--no-cri", "--pmc", "--plugin-dir", FAKE_DIR, "--log-level", "error"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=e, text=True)
    try:
        kids = []
        for _ in range(50):
            time.sleep(0.1)
            kids = [int(k) for t in os.listdir(f"/proc/{p.pid}/task")
                    for k in open(f"/proc/{p.pid}/task/{t}/children").read().split()]
            if kids:
                break
        assert len(kids) == 1
        status = dict(l.split(":", 1) for l in open(f"/proc/{kids[0]}/status") if ":" in l)
        assert int(status["SigBlk"].strip(), 16) == 0, status["SigBlk"]
    finally:
        p.terminate()
        p.wait(20)


def test_own_helper_is_not_a_workload_or_a_sharer(core, mock_exporter, monkeypatch):
    """The exporter's on-device helper holds a GPU context on every device and (with --probe) runs
    the K1 probe's waves. Its KFD process entry must not become a pod_gpu row, count toward
    gpu_active_processes, or make an exclusively used GPU look shared (which would withdraw the
    tenant's pod_gpu_mfma_util_percent)."""
    monkeypatch.setenv("GPUMON_FAKE_AGENTS", "1")
    ex = mock_exporter(backend="mock:gpus=1,mode=idle", sample_threads=0)
    od = _ondevice(core, ex, ondevice_isolate=True)
    od.start()
    try:
        assert od.step()
        helper = core.ondevice_helper_pid()
        assert helper > 0
        ex.mock_set_procs([{"pid": 4242, "device": 0, "name": "train", "kfd_only": True},
                           {"pid": helper, "device": 0, "name": "gpumon-ondevice", "kfd_only": True}])
        ex.mock_set_occ_series(0, [200.0, 8.0])  # both have waves resident (the helper: the probe)
        ex.set_device_mfma_util({0: 61.0})
        ex.tick()
        rows = [r for r in ex.pod_rows() if not r["idle"]]
        assert [r["pid"] for r in rows] == ["4242"] and rows[0]["mfma_util"] is not None
        m = ex.metrics_text()
        assert _val(m, "gpu_active_processes", gpu_id="0") == 1
        assert "gpumon_ondevice_helper_gpu_contexts" in m and f'pid="{helper}"' not in m
    finally:
        od.stop()


def test_helper_checks_its_parent_by_pid():
    """the helper used `getppid() == 1` as "parent already gone" -- always true when the
    exporter is PID 1 itself (ENTRYPOINT without hostPID), so PMC and probe never started there. The
    exporter now passes its pid; the helper exits only if its parent is not that process."""
    import time

    helper = os.path.join(FAKE_DIR, "gpumon-ondevice-helper")
    gone = subprocess.Popen([helper, "--parent-pid=1"], stdin=subprocess.PIPE, stdout=subprocess.PIPE)
    assert gone.wait(10) == 0  # its parent (this process) is not pid 1's stand-in: already gone
    alive = subprocess.Popen([helper, f"--parent-pid={os.getpid()}"], stdin=subprocess.PIPE, stdout=subprocess.PIPE)
    try:
        time.sleep(0.5)
        assert alive.poll() is None  # parent matches: serves requests
    finally:
        alive.stdin.close()  # EOF on the request pipe: clean exit
        assert alive.wait(10) == 0
