"""PMC (rocprofiler-sdk device counting) on a real MI355X, in a fresh subprocess because the tool
must register before HSA initialises. MFMA-busy must separate idle / bf16 burn / HBM stream."""

import json
import os
import subprocess
import sys

import pytest


pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pmc_separates_idle_mfma_hbm():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools/pmc_check.py")], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["agents"][0]["cu_count"] == 256 and d["agents"][0]["num_xcc"] == 8
    assert d["idle"].get("mfma_busy", 0) < 5
    assert d["mfma"]["mfma_busy"] > 60, d["mfma"]
    assert d["hbm"].get("mfma_busy", 0) < 5
    assert d["hbm"]["occupancy"] > 20
    assert d["mfma"]["gui_active"] > 90
    # achieved bf16 MFMA throughput from SQ_INSTS_VALU_MFMA_MOPS_BF16 (LoadGen reports ~2 PFLOP/s)
    assert 1000 < d["mfma"]["mfma_tflops"]["bf16"] < 2600, d["mfma"]
    assert d["idle"].get("mfma_tflops", {}).get("bf16", 0) < 5 and d["hbm"]["mfma_tflops"]["bf16"] < 5
    tf_load = d["mfma_load"]["tflops"]
    assert abs(d["mfma"]["mfma_tflops"]["bf16"] - tf_load) < 0.25 * tf_load, (d["mfma"], tf_load)
    # partial occupancy (burn on ~1/4 of the CUs): busy GPU, but MFMA pipes mostly idle
    assert 5 < d["partial"]["mfma_busy"] < 0.6 * d["mfma"]["mfma_busy"], d["partial"]
    assert len(d["mfma"].get("xcd_mfma_busy", [])) == 8
    assert d["mfma_many"][0]["mfma_busy"] > 60, d["mfma_many"]  # sample_many agrees with sample
    print("pmc:", {k: d[k] for k in ("idle", "mfma", "hbm")})


def test_mfma_tflops_per_dtype_match_events():
    """gpu_mfma_tflops{dtype}: each matrix path's burn lights exactly its own MOPS counter, at the
    event-timed rate (profiles/r1_mfma_dtypes.md)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools/mfma_dtypes.py"), "fp8", "mxfp4", "i8", "f64"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    want = {"fp8": "f8", "mxfp4": "f6f4", "i8": "i8", "f64": "f64"}
    for dt, counter in want.items():
        (got, tf), = d[dt]["pmc_tflops"].items()
        assert got == counter, d[dt]
        ev = d[dt]["event_tflops"]
        assert abs(tf - ev) < 0.03 * ev, d[dt]
    assert d["mxfp4"]["event_tflops"] > 3 * d["fp8"]["event_tflops"]  # the 4x-rate f8f6f4 path
