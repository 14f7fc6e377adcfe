"""Golden exposition (SURVEY.md §4.2 "schema + rendering: unit + golden"): two ticks of the REAL
amdsmi backend against the deterministic fake libamd_smi (csrc/fakes/fake_amd_smi.cpp) with an
empty procfs, rendered to Prometheus text and to Influx line protocol, compared byte-for-byte
with tests/golden/ after dropping the exporter's own timing/self metrics and line timestamps.

Regenerate after an intended schema change:  GPUMON_UPDATE_GOLDEN=1 pytest tests/test_golden.py
"""

import os
import re

import pytest

from conftest import make_locked

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(ROOT, "build", "fakes", "libfake_amd_smi.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")
VOLATILE = re.compile(r"^(# (HELP|TYPE) )?(gpumon_|process_)")


@pytest.fixture(scope="module", autouse=True)
def fake_lib():
    make_locked("fakes")


def _exporter(core, monkeypatch, tmp_path):
    for k in ("FAKE_AMDSMI_GPUS", "FAKE_AMDSMI_PROCS", "FAKE_AMDSMI_CPX", "FAKE_AMDSMI_NO_METRICS",
              "FAKE_AMDSMI_FAIL_METRICS", "FAKE_AMDSMI_INIT_FAIL"):
        monkeypatch.delenv(k, raising=False)
    (tmp_path / "proc").mkdir()
    ex = core.Exporter({"backend": "amdsmi", "amdsmi_lib": FAKE, "serve_http": False, "interval_s": 0,
                        "host": "golden-node", "verify_kfd": False, "init_retry_s": 0.0, "fast_path": False,
                        "procfs_root": str(tmp_path / "proc"), "sample_threads": 0})
    assert ex.start() == ""
    return ex


def _check(name, text):
    path = os.path.join(GOLDEN, name)
    if os.environ.get("GPUMON_UPDATE_GOLDEN"):
        with open(path, "w") as f:
            f.write(text)
    with open(path) as f:
        want = f.read()
    assert text == want, f"{name} differs from the golden file (GPUMON_UPDATE_GOLDEN=1 to accept)"


def test_prometheus_golden(core, monkeypatch, tmp_path):
    ex = _exporter(core, monkeypatch, tmp_path)
    try:
        ex.tick()
        ex.tick()
        text = "".join(l + "\n" for l in ex.metrics_text().splitlines() if not VOLATILE.match(l))
    finally:
        ex.stop()
    _check("fake_amdsmi_2ticks.prom", text)


def test_influx_golden(core, monkeypatch, tmp_path):
    ex = _exporter(core, monkeypatch, tmp_path)
    try:
        ex.tick()
        ex.tick()
        lines = [re.sub(r" \d{19}$", " <ts>", l) for l in ex.influx_text().splitlines()]
    finally:
        ex.stop()
    _check("fake_amdsmi_2ticks.influx", "".join(l + "\n" for l in lines))
