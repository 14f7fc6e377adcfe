"""A tenant profiling its own job with `rocprofv3 --pmc` while the exporter's continuous device
counting runs on the same GPU (SQ/GRBM counters are a shared device resource). Required: the
tenant's profile completes with sane counters, the exporter survives, and it never exports
garbage -- either its MFMA series stay within bounds or it flags the conflict (gpumon_pmc_up 0,
gpumon_pmc_errors_total / gpumon_pmc_resets_total). The reference's shared channel was nvidia-smi
(/root/reference/gpu.py:104-116)."""

import csv
import glob
import os
import socket
import subprocess
import sys
import tempfile
import time
import urllib.request

import pytest

from gpumon.export import promtext

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scrape(port):
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
        return promtext.parse(r.read().decode())


def test_tenant_rocprofv3_pmc_while_exporter_counts():
    port = _port()
    exe = os.path.join(ROOT, "bin", "gpumon-exporter")
    ex = subprocess.Popen([exe, "--backend", "amdsmi", "--interval", "0.2", "--pmc", "--listen",
                           f"127.0.0.1:{port}", "--log-level", "warn", "--no-pod-resources", "--no-cri"],
                          stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    out = tempfile.mkdtemp(prefix="gpumon-coexist-", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        time.sleep(3)
        assert ex.poll() is None, ex.stderr.read()[-2000:]
        before = _scrape(port)
        assert promtext.one(before, "gpumon_pmc_up") == 1
        env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
        r = subprocess.run(["rocprofv3", "--pmc", "SQ_WAVES", "GRBM_GUI_ACTIVE", "--kernel-trace", "-f", "csv",
                            "-d", out, "-o", "run", "--", sys.executable, "-m", "gpumon", "load", "--kind", "mfma",
                            "--seconds", "4"], capture_output=True, text=True, timeout=100, cwd=ROOT, env=env)
        during = _scrape(port)
        time.sleep(1.0)
        after = _scrape(port)
        assert ex.poll() is None, "exporter died: " + ex.stderr.read()[-2000:]
        # the tenant's profile completed with sane counters
        assert r.returncode == 0, r.stderr[-3000:]
        files = glob.glob(os.path.join(out, "**", "*counter_collection*.csv"), recursive=True)
        assert files, os.listdir(out)
        rows = list(csv.DictReader(open(files[0])))
        waves = [float(x["Counter_Value"]) for x in rows if x.get("Counter_Name") == "SQ_WAVES"]
        assert waves and max(waves) > 0, rows[:3]
        # the exporter never exported garbage
        for fam in (during, after):
            for v in promtext.values(fam, "gpu_mfma_util_percent") + promtext.values(fam, "gpu_mfma_busy_active_percent"):
                assert 0 <= v <= 100, v
        assert promtext.one(after, "gpumon_pmc_up") in (0, 1)
        print("coexist: pmc_up during/after", promtext.one(during, "gpumon_pmc_up"), promtext.one(after, "gpumon_pmc_up"),
              "errors", promtext.one(after, "gpumon_pmc_errors_total"),
              "resets", promtext.one(after, "gpumon_pmc_resets_total"))
    finally:
        ex.terminate()
        try:
            ex.wait(20)
        except subprocess.TimeoutExpired:
            ex.kill()
            ex.wait(10)
