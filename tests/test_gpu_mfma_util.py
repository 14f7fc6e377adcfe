"""End-to-end wall-time MFMA utilisation of the deployed exporter (bin/gpumon-exporter --pmc: the
on-device helper, continuous counting, gpu_mfma_util_percent) against the event-timed duty of a
tenant process on a real MI355X. Round-1 VERDICT item 4: within 5 points, including a
150 ms on / 150 ms off burst pattern (the windowed sampler aliased such bursts)."""

import json
import os
import socket
import statistics
import subprocess
import sys
import time
import urllib.request

import pytest

from gpumon.export import promtext

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(port, load_args, seconds):
    """Median exported MFMA util over the ticks fully inside the load, and the load's busy share."""
    load = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mfma", "--seconds", str(seconds),
                             *load_args], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
    vals, pod = [], []
    t_end = time.time() + seconds
    time.sleep(2.5)  # load running, two full ticks since its start
    while time.time() < t_end - 1.2:
        m = urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5).read().decode()
        fam = promtext.parse(m)
        v = promtext.values(fam, "gpu_mfma_util_percent", gpu_id="0")
        if v:
            vals.append(v[0])
            pod.append((v[0], promtext.values(fam, "pod_gpu_mfma_util_percent", gpu_id="0")))
        time.sleep(1.0)
    out, _ = load.communicate(timeout=120)
    st = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    busy = st["busy_s"] / st["wall_s"]
    return statistics.median(vals), busy, vals, pod


def test_exported_mfma_util_tracks_duty_and_bursts():
    port = _port()
    ex = subprocess.Popen([os.path.join(ROOT, "bin", "gpumon-exporter"), "--backend", "amdsmi", "--interval", "1",
                           "--pmc", "--probe", "--listen", f"127.0.0.1:{port}", "--no-pod-resources", "--no-cri",
                           "--log-level", "warn"], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(3)
        assert ex.poll() is None, ex.stderr.read()[-2000:]
        full, busy_full, _, pod = _run(port, [], 9)
        assert full > 60, full
        # the tenant is the GPU's only process with waves: its row carries the device's MFMA util
        # (the two series come from the same snapshot; a tick can fall between PMC updates). The
        # helper's K1 probe waves (--probe) do not make the GPU look shared.
        assert sum(1 for dev, rows in pod if len(rows) == 1 and abs(rows[0] - dev) < 10) >= len(pod) - 1, pod
        rows = {}
        for name, args in (("duty50", ["--duty", "0.5"]), ("burst150ms", ["--duty", "0.5", "--period", "0.3"])):
            got, busy, vals, _ = _run(port, args, 10)
            want = full * busy / busy_full
            rows[name] = (round(got, 1), round(want, 1), [round(v, 1) for v in vals])
            print(f"\n{name}: exported {got:.1f} %, event-timed expectation {want:.1f} % (busy {busy:.3f})")
        for name, (got, want, vals) in rows.items():
            assert abs(got - want) <= 5.0, (name, rows)
    finally:
        ex.terminate()
        ex.wait(20)
