"""ROCTx ranges around sampler phases (SURVEY.md §5 tracing row): off by default (no library
loaded, no ranges), and when enabled every tick opens tick/sample/sample_dev/attrib/render/gzip
ranges (gzip only while scrapes keep asking for it). librocprofiler-sdk-roctx ships in the ROCm image, so this runs on CPU too."""

import os

import pytest


def test_roctx_ranges_bracket_each_tick(core):
    if not os.path.exists("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"):
        pytest.skip("no roctx library")
    ex = core.Exporter({"backend": "mock:gpus=2", "serve_http": False, "interval_s": 0, "roctx": True})
    ex.start()
    try:
        assert core.roctx_active()
        r0 = core.roctx_ranges()
        ex.tick()
        # tick + sample + 2 x sample_dev + attrib + render; no gzip range: nobody scraped with gzip,
        # so the tick thread does not compress (Snapshot::gzipped, lazy until scrapes ask for it)
        assert core.roctx_ranges() - r0 == 6
    finally:
        ex.stop()
        core.roctx_enable(False)
    r1 = core.roctx_ranges()
    ex2 = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0})
    ex2.start()
    ex2.tick()
    ex2.stop()
    assert core.roctx_ranges() == r1  # disabled: no ranges


def test_config_roctx_flag():
    import argparse

    from gpumon.config import Config, add_cli_args, from_args

    def parse(argv, env):
        p = argparse.ArgumentParser()
        add_cli_args(p)
        return from_args(p.parse_args(argv), env=env)

    assert Config().roctx is False
    assert parse(["--roctx"], {}).roctx is True
    assert parse([], {"GPUMON_ROCTX": "1"}).roctx is True
