from gpumon.config import Config
from gpumon.ops.pmc import DEFAULT_COUNTERS


def test_config_pmc_counters_cover_derivations():
    assert set(DEFAULT_COUNTERS) <= set(Config().pmc_counters)
