"""The K1 probe's two launch paths on the MI355X (lib/libgpumon_probe.so; profiles/r3_probe_hsa.md):
raw AQL dispatch on one HSA queue (the default) and a HIP stream, each in a process of its own.
Both must see every XCD and CU with no stale record; the HSA path must not carry the HIP runtime
(smaller process) and its kernel arguments must stay L2-cacheable (wave spread near HIP's, not the
~28 us of host-memory kernargs read by every CU)."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hsa_and_hip_probe_paths_agree():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "probe_runtime_check.py"), "--launches", "50"],
                       capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rows = {d["runtime"]: d for d in map(json.loads, r.stdout.strip().splitlines())}
    assert set(rows) == {"hsa", "hip"}, rows
    for rt, d in rows.items():
        assert "error" not in d, (rt, d)
        assert d["complete"] == 50 and d["stale_records"] == 0, (rt, d)
        assert d["min_blocks_per_xcd"] >= 100 and d["unique_cus"] >= 250, (rt, d)
        assert all(1500 < c < 2600 for c in d["xcd_clock_mhz_last"]), (rt, d)
    hsa, hip = rows["hsa"], rows["hip"]
    assert hsa["rss_mb"] < hip["rss_mb"] - 50, (hsa, hip)  # no HIP runtime in the HSA process
    assert hsa["kernel_span_us_p50"] < 15, hsa  # coarse-grained (L2-cached) kernargs
    assert hsa["create_ms"] < hip["create_ms"], (hsa, hip)
