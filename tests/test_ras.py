"""RAS / ECC counters (csrc/core/ras.cpp): the kernel's ras/ sysfs files (aca_<block> on MI355X,
legacy <block>_err_count, event_state, gpu_vram_bad_pages), the per-block amdsmi fallback, the
refresh cadence with carry-over, and the mock's fault injection. The on-box file layout was
measured on MI355X (profiles/r1_ras.md)."""


import pytest

from conftest import make_locked
from gpumon.export import promtext
from test_sysfs_fast import FAKE, make_tree

MI355X_EVENT_STATE = ("current seqno: 7\nFatal Error: count:1, last_seqno:3\n"
                      "Poison Creation: count:2, last_seqno:5\nPoison Consumption: count:4, last_seqno:7\n")


@pytest.fixture(scope="module", autouse=True)
def fakes():
    make_locked("fakes")


def _ras_dir(sysr, d=0):
    r = sysr / "bus" / "pci" / "devices" / f"0000:{0x26 + 0x20 * d:02x}:00.0" / "ras"
    r.mkdir(parents=True, exist_ok=True)
    return r


def _exporter(core, monkeypatch, sysr, procr, env=None, **over):
    for k in ("FAKE_AMDSMI_GPUS", "FAKE_AMDSMI_CPX", "FAKE_AMDSMI_NO_METRICS", "FAKE_AMDSMI_ECC_UMC_CE",
              "FAKE_AMDSMI_BAD_PAGES"):
        monkeypatch.delenv(k, raising=False)
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, str(v))
    cfg = {"backend": "amdsmi", "amdsmi_lib": FAKE, "serve_http": False, "interval_s": 0, "host": "n1",
           "verify_kfd": False, "init_retry_s": 0.0, "sysfs_root": str(sysr), "procfs_root": str(procr)}
    cfg.update(over)
    ex = core.Exporter(cfg)
    assert ex.start() == ""
    return ex


def test_sysfs_aca_files(core, monkeypatch, tmp_path):
    sysr, procr = make_tree(tmp_path)
    r = _ras_dir(sysr)
    (r / "aca_umc").write_text("ue: 1\nce: 12\nde: 3\n")
    (r / "aca_gfx").write_text("ue: 0\nce: 5\nde: 0\n")
    (r / "aca_xgmi_wafl").write_text("ue: 0\nce: 0\nde: 0\n")
    (r / "umc_err_count").write_text("ue: 99\nce: 99\n")  # legacy duplicate: the ACA file wins
    (r / "event_state").write_text(MI355X_EVENT_STATE)
    (r / "gpu_vram_bad_pages").write_text("0x00001234 : 0x00001000 : R\n0x00005678 : 0x00001000 : P\n")
    (r / "features").write_text("feature mask: 0x400fdbff\n")
    ex = _exporter(core, monkeypatch, sysr, procr)
    try:
        ex.tick()
        s = ex.samples()
        assert s[0]["ras"]["source"] == "sysfs"
        assert s[0]["ras"]["blocks"]["umc"] == {"ue": 1, "ce": 12, "de": 3}
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpu_ecc_errors_total", gpu_id="0", block="umc", type="uncorrectable") == 1
        assert promtext.one(fam, "gpu_ecc_errors_total", gpu_id="0", block="umc", type="correctable") == 12
        assert promtext.one(fam, "gpu_ecc_errors_total", gpu_id="0", block="umc", type="deferred") == 3
        assert promtext.one(fam, "gpu_ecc_errors_total", gpu_id="0", block="gfx", type="correctable") == 5
        assert promtext.one(fam, "gpu_ras_events_total", gpu_id="0", event="fatal") == 1
        assert promtext.one(fam, "gpu_ras_events_total", gpu_id="0", event="poison_creation") == 2
        assert promtext.one(fam, "gpu_ras_events_total", gpu_id="0", event="poison_consumption") == 4
        assert promtext.one(fam, "gpu_retired_pages", gpu_id="0") == 2
        # device 1 has no ras/ directory: amdsmi per-block fallback (5 blocks answer, as on MI355X)
        assert s[1]["ras"]["source"] == "amdsmi"
        assert sorted(s[1]["ras"]["blocks"]) == ["gfx", "mmhub", "sdma", "umc", "xgmi_wafl"]
        assert "ras" in ex.self_stats()["backend_calls"]
    finally:
        ex.stop()


def test_legacy_err_count_files_without_deferred(core, monkeypatch, tmp_path):
    sysr, procr = make_tree(tmp_path, gpus=1)
    r = _ras_dir(sysr)
    (r / "umc_err_count").write_text("ue: 2\nce: 7\n")
    (r / "sdma_err_count").write_text("ue: 0\nce: 1\n")
    ex = _exporter(core, monkeypatch, sysr, procr, env={"FAKE_AMDSMI_GPUS": 1})
    try:
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpu_ecc_errors_total", block="umc", type="uncorrectable") == 2
        assert promtext.one(fam, "gpu_ecc_errors_total", block="sdma", type="correctable") == 1
        assert not promtext.values(fam, "gpu_ecc_errors_total", type="deferred")
        assert not promtext.values(fam, "gpu_ras_events_total")  # no event_state file
    finally:
        ex.stop()


def test_amdsmi_fallback_counts_and_bad_pages(core, monkeypatch, tmp_path):
    sysr, procr = make_tree(tmp_path, gpus=1)
    ex = _exporter(core, monkeypatch, sysr, procr, env={"FAKE_AMDSMI_GPUS": 1, "FAKE_AMDSMI_ECC_UMC_CE": 6,
                                                         "FAKE_AMDSMI_BAD_PAGES": 3})
    try:
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpu_ecc_errors_total", block="umc", type="correctable") == 6
        assert promtext.one(fam, "gpu_retired_pages", gpu_id="0") == 3
        assert len(promtext.values(fam, "gpu_ecc_errors_total")) == 5 * 3
        st = ex.self_stats()["backend_calls"]["ras"]
        assert st["errors"] == 0  # the blocks MI355X does not track were dropped, not counted as errors
    finally:
        ex.stop()


def test_refresh_cadence_and_carry_over(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=2", ras_every=3)
    ex.mock_add_ecc(1, "umc", ue=0, ce=4)
    seen = []
    for _ in range(6):
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        seen.append(promtext.values(fam, "gpu_ecc_errors_total", gpu_id="1", block="umc", type="correctable"))
    # refreshed once within 3 ticks, then carried over on the ticks between refreshes (never missing)
    first = next(i for i, v in enumerate(seen) if v == [4.0])
    assert first < 3 and all(v == [4.0] for v in seen[first:]), seen
    assert all(v in ([0.0], [4.0]) for v in seen)
    ex.mock_add_ecc(0, "umc", ue=1)
    ex.mock_set_ras_event(0, "poison_consumed", 2)
    ex.mock_set_ras_event(0, "bad_pages", 9)
    for _ in range(4):  # read within ras_every ticks, exported on the tick after (ras_async)
        ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpu_ecc_errors_total", gpu_id="0", block="umc", type="uncorrectable") == 1
    assert promtext.one(fam, "gpu_ras_events_total", gpu_id="0", event="poison_consumption") == 2
    assert promtext.one(fam, "gpu_retired_pages", gpu_id="0") == 9
    assert promtext.one(fam, "gpu_ecc_errors_total", gpu_id="1", block="umc", type="correctable") == 4


def test_ras_off(mock_exporter):
    ex = mock_exporter(ras_every=0)
    ex.tick()
    ex.tick()
    text = ex.metrics_text()
    assert "gpu_ecc_errors_total" not in text and "gpu_retired_pages" not in text


def test_sysfs_refresh_can_be_spread_over_ras_slices_ticks(core, monkeypatch, tmp_path):
    """A full pass over the ras/ files costs 0.25-0.5 ms on MI355X; with ras_slices = ras_every each
    tick re-reads one slice (file index mod ras_slices) and keeps the rest from the last pass, so no
    tick pays for all of them and every counter is at most ras_every ticks old."""
    sysr, procr = make_tree(tmp_path, gpus=1)
    r = _ras_dir(sysr)
    (r / "aca_gfx").write_text("ue: 0\nce: 1\nde: 0\n")      # item 0
    (r / "aca_umc").write_text("ue: 0\nce: 2\nde: 0\n")      # item 1
    (r / "aca_xgmi_wafl").write_text("ue: 0\nce: 0\nde: 0\n")  # item 2
    (r / "event_state").write_text(MI355X_EVENT_STATE)      # item 3
    ex = _exporter(core, monkeypatch, sysr, procr, env={"FAKE_AMDSMI_GPUS": 1}, ras_every=3, ras_slices=3)

    def ce():
        b = ex.samples()[0]["ras"]["blocks"]
        return b["gfx"]["ce"], b["umc"]["ce"], sorted(b)

    try:
        ex.tick()  # first tick: everything
        assert ce() == (1, 2, ["gfx", "umc", "xgmi_wafl"])
        (r / "aca_gfx").write_text("ue: 0\nce: 10\nde: 0\n")
        (r / "aca_umc").write_text("ue: 0\nce: 20\nde: 0\n")
        seen = []
        for _ in range(4):
            ex.tick()
            seen.append(ce())
        assert all(s[2] == ["gfx", "umc", "xgmi_wafl"] for s in seen)  # never a partial block set
        assert seen[-1][:2] == (10, 20)  # both read within ras_every ticks (exported the tick after) ...
        assert any(s[:2] in ((10, 2), (1, 20)) for s in seen), seen  # ... on different ticks
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpu_ras_events_total", event="poison_consumption") == 4  # carried
    finally:
        ex.stop()


def test_ras_pass_runs_on_one_tick_per_ras_every_by_default(mock_exporter):
    """ras_slices = 1 (default): the whole pass on one tick out of every ras_every (one firmware
    query burst per GPU per period), staggered across GPUs; ras_slices = N spreads it over N
    consecutive ticks."""
    ex = mock_exporter(backend="mock:gpus=2", ras_every=4)
    for _ in range(9):
        ex.tick()
    log = ex.tick_log()
    assert log[0]["ras_reads"] == 2 and log[0]["ras_full"]  # first tick: every GPU, everything
    # ticks 1..8: each GPU reads once per 4 ticks, never both on the same tick (staggered)
    assert [t["ras_reads"] for t in log[1:9]] == [0, 0, 1, 1, 0, 0, 1, 1]
    ex2 = mock_exporter(backend="mock:gpus=1", ras_every=4, ras_slices=2)
    for _ in range(9):
        ex2.tick()
    reads = [t["ras_reads"] for t in ex2.tick_log()[1:9]]
    assert reads == [1, 0, 0, 1, 1, 0, 0, 1] and not ex2.tick_log()[1]["ras_full"]


def test_failed_ras_read_keeps_last_values_and_is_reported(core, monkeypatch, tmp_path):
    """A due file that fails to read keeps its last value (event_state, bad pages included: the
    series never blank for a cycle) and the RAS call counts as failed, so a stuck file shows in
    gpumon_backend_call_errors_total{call="ras"} instead of freezing silently."""
    sysr, procr = make_tree(tmp_path, gpus=1)
    r = _ras_dir(sysr)
    (r / "aca_umc").write_text("ue: 0\nce: 2\nde: 0\n")
    (r / "event_state").write_text(MI355X_EVENT_STATE)
    ex = _exporter(core, monkeypatch, sysr, procr, env={"FAKE_AMDSMI_GPUS": 1}, ras_every=1)
    try:
        ex.tick()
        assert ex.self_stats()["backend_calls"]["ras"]["errors"] == 0
        (r / "event_state").unlink()
        (r / "event_state").mkdir()  # unreadable as a file (root ignores permission bits)
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpu_ras_events_total", event="poison_consumption") == 4  # carried
        assert promtext.one(fam, "gpu_ecc_errors_total", block="umc", type="correctable") == 2
        assert ex.self_stats()["backend_calls"]["ras"]["errors"] == 1
    finally:
        ex.stop()


def test_async_ras_is_off_the_tick_path(mock_exporter):
    """ras_async (default): the device worker reads the RAS slice after publishing the tick, so
    the RAS tick costs no more than the others and its values arrive on the next tick."""
    ex = mock_exporter(backend="mock:gpus=1", ras_every=1)
    ex.mock_add_ecc(0, "umc", ue=2)
    ex.tick()  # reads (asynchronously) the new count
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpu_ecc_errors_total", block="umc", type="uncorrectable") == 0  # not yet
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpu_ecc_errors_total", block="umc", type="uncorrectable") == 2
    sync = mock_exporter(backend="mock:gpus=1", ras_every=1, ras_async=False)
    sync.mock_add_ecc(0, "umc", ue=3)
    sync.tick()
    fam = promtext.parse(sync.metrics_text())
    assert promtext.one(fam, "gpu_ecc_errors_total", block="umc", type="uncorrectable") == 3


@pytest.mark.parametrize("backend", ["amdsmi", "rocm_smi"])
def test_transient_first_read_failure_does_not_switch_ras_off(core, monkeypatch, tmp_path, backend):
    """a first pass whose listed files could not be read (empty cache, a file briefly
    unreadable) latched the device's sysfs RAS off until re-init -- the amdsmi backend then fell
    back to library ECC calls for good, the rocm_smi one stopped reading RAS at all. Only a
    directory without error-count files may do that; a transient failure is retried with backoff."""
    from test_rocm_smi_fake import FAKE_RSMI

    sysr, procr = make_tree(tmp_path, gpus=1)
    r = _ras_dir(sysr)
    (r / "aca_umc").mkdir()  # listed, but reading it fails (EISDIR) on the first pass
    over = {"ras_every": 1, "ras_async": False}
    if backend == "rocm_smi":
        over.update(backend="rocm_smi", rocm_smi_lib=FAKE_RSMI)
    ex = _exporter(core, monkeypatch, sysr, procr, env={"FAKE_AMDSMI_GPUS": 1, "FAKE_RSMI_GPUS": 1}, **over)
    try:
        ex.tick()
        assert ex.self_stats()["backend_calls"]["ras"]["errors"] >= 1
        (r / "aca_umc").rmdir()
        (r / "aca_umc").write_text("ue: 0\nce: 9\nde: 0\n")
        for _ in range(3):  # one pass skipped (backoff), then read again
            ex.tick()
        s = ex.samples()[0]["ras"]
        assert s["source"] == "sysfs" and s["blocks"]["umc"]["ce"] == 9, s
    finally:
        ex.stop()


def test_ras_retry_backoff_is_bounded(core, monkeypatch, tmp_path):
    """Files that stay unreadable are retried ever more rarely (skip 1, 3, 7, ... 63 passes)."""
    sysr, procr = make_tree(tmp_path, gpus=1)
    r = _ras_dir(sysr)
    (r / "aca_umc").mkdir()
    ex = _exporter(core, monkeypatch, sysr, procr, env={"FAKE_AMDSMI_GPUS": 1}, ras_every=1, ras_async=False)
    try:
        for _ in range(40):
            ex.tick()
        st = ex.self_stats()["backend_calls"]["ras"]
        assert 3 <= st["n"] <= 6, st  # passes at ticks 0, 2, 6, 14, 30 -- not 40
        assert (ex.samples()[0]["ras"] or {}).get("source") != "amdsmi"  # never latched to the fallback
    finally:
        ex.stop()
