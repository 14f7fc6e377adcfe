"""CPU unit test of the PMC derivation formulas (gfx9xx fallbacks used for gfx950)."""

import pytest

from oracles.ops.pmc import derive

AGENT = {"cu_count": 256, "simd_count": 1024, "max_waves_per_cu": 32}


def test_full_mfma():
    raw = {"GRBM_GUI_ACTIVE": {"sum": 8e6, "max": 1e6}, "GRBM_COUNT": {"max": 1e6},
           "SQ_VALU_MFMA_BUSY_CYCLES": {"sum": 1024e6, "by_xcc": [128e6] * 8}, "SQ_WAVE_CYCLES": {"sum": 256e6 * 8 / 4}}
    d = derive(raw, AGENT)
    assert d["mfma_busy"] == pytest.approx(100.0)
    assert d["xcd_mfma_busy"] == pytest.approx([100.0] * 8)
    assert d["occupancy"] == pytest.approx(400 * 512e6 / 1e6 / 256 / 32)
    assert d["gui_active"] == pytest.approx(100.0)


def test_idle_and_missing():
    assert derive({"GRBM_GUI_ACTIVE": {"max": 0.0}}, AGENT) == {}
    assert derive({}, AGENT) == {}


def test_config_pmc_counters_cover_derivations():
    """The default counter set (one gfx950 counting pass) holds every counter derive() uses."""
    from gpumon.config import Config
    from oracles.ops.pmc import DEFAULT_COUNTERS

    assert set(DEFAULT_COUNTERS) <= set(Config().pmc_counters)
    assert Config().pmc_mode == "continuous"
