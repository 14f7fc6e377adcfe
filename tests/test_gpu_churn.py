"""Process churn on the real GPU (tools/churn_soak.py, profiles/r3_churn.md): tenants with their
own HIP contexts start and exit while the exporter samples at 10 Hz; every tenant the KFD shows
holding VRAM gets a row, no row outlives its process, nothing is left after the last exit. The
reference rebuilt its process list every cycle with `docker top` (/root/reference/gpu.py:174-178);
the exporter keeps per-pid state across ticks, which churn must not corrupt or leak."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rows_follow_arriving_and_departing_tenants():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tools", "churn_soak.py"), "--minutes", "0.5",
                        "--window", "10", "--max-tenants", "4", "--grace", "3", "--seed", "5"],
                       capture_output=True, text=True, timeout=150, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    s = json.loads(r.stdout.strip().splitlines()[-1])
    assert s["tenants_started"] >= 5 and s["tenants_failed"] == 0, s
    assert s["rows_max"] >= 1, s
    assert s["missed"] == 0 and s["stale"] == 0, s
    assert s["rows_left_after_drain"] == [] and s["drained"], s
    assert s["overruns"] == 0 and s["device_errors"] == 0 and s["scrape_errors"] == 0, s
