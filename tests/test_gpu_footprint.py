"""The exporter stays inside the DaemonSet's requests / limits on an MI355X (profiles/
r2_footprint.md). Measured in the deployed shape: the exporter (and, with PMC, its frozen helper
process) next to a separate load process. The reference set no limits at all
(/root/reference/gpu_monitor.yaml:21-37)."""

import os
import socket
import subprocess
import sys
import time

import pytest
import yaml

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HZ = os.sysconf("SC_CLK_TCK")


def _mem_mib(q):
    return float(q[:-2]) * (1024 if q.endswith("Gi") else 1) if q.endswith(("Mi", "Gi")) else float(q) / 2 ** 20


def _limits(path, patched=False):
    docs = [d for d in yaml.safe_load_all(open(os.path.join(ROOT, path))) if d]
    if patched:
        (k,) = docs
        res = next(yaml.safe_load(p["patch"])[0]["value"] for p in k["patches"] if p["target"]["kind"] == "DaemonSet")
    else:
        ds = next(d for d in docs if d["kind"] == "DaemonSet")
        res = ds["spec"]["template"]["spec"]["containers"][0]["resources"]
    cpu_m = float(res["requests"]["cpu"].rstrip("m"))
    return cpu_m, _mem_mib(res["limits"]["memory"])


def _tree(pid):
    pids = [pid] + [int(p) for p in os.listdir("/proc") if p.isdigit() and _ppid(p) == pid]
    rss = cpu = 0.0
    for p in pids:
        try:
            for line in open(f"/proc/{p}/status"):
                if line.startswith("VmRSS:"):
                    rss += int(line.split()[1]) / 1024
            f = open(f"/proc/{p}/stat").read().rsplit(")", 1)[1].split()
            cpu += (int(f[11]) + int(f[12])) / HZ
        except OSError:
            pass
    return rss, cpu


def _ppid(p):
    try:
        return int(open(f"/proc/{p}/stat").read().rsplit(")", 1)[1].split()[1])
    except (OSError, ValueError, IndexError):
        return -1


def _measure(flags, seconds=10.0, python=False):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    if python:  # the DaemonSet's entrypoint (deploy/Dockerfile): python3 -m gpumon serve
        cmd = [sys.executable, "-m", "gpumon", "serve", "--backend", "amdsmi", "--listen", f"127.0.0.1:{port}",
               "--log-level", "warn", "--control-plane", "off", *flags]
    else:
        cmd = [os.path.join(ROOT, "bin", "gpumon-exporter"), "--backend", "amdsmi", "--listen", f"127.0.0.1:{port}",
               "--log-level", "warn", "--no-pod-resources", "--no-cri", *flags]
    ex = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(8)  # start-up (HSA / rocprofiler init) is not steady state
        assert ex.poll() is None, ex.stderr.read()[-2000:]
        _, c0 = _tree(ex.pid)
        t0 = time.time()
        rss = 0.0
        while time.time() - t0 < seconds:
            rss = max(rss, _tree(ex.pid)[0])
            time.sleep(1.0)
        _, c1 = _tree(ex.pid)
        return 1000 * (c1 - c0) / (time.time() - t0), rss
    finally:
        ex.terminate()
        ex.wait(20)


@pytest.fixture(scope="module")
def load():
    p = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mixed", "--seconds", "60"], cwd=ROOT,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    time.sleep(4)
    yield p
    p.terminate()
    p.wait(60)


@pytest.mark.parametrize("python", [False, True], ids=["native", "serve"])
def test_default_exporter_within_daemonset_limits(load, python):
    cpu_req, mem_lim = _limits("deploy/k8s/gpumon-daemonset.yaml")
    mcores, rss = _measure(["--interval", "1"], python=python)
    print(f"\ndefault: {mcores:.1f} millicores, {rss:.1f} MiB (request {cpu_req}m, limit {mem_lim} MiB)")
    assert mcores < cpu_req and rss < mem_lim / 4


@pytest.mark.parametrize("python", [False, True], ids=["native", "serve"])
def test_ondevice_exporter_within_overlay_limits(load, python):
    cpu_req, mem_lim = _limits("deploy/k8s/overlays/ondevice/kustomization.yaml", patched=True)
    flags = ["--interval", "1"] + (["--enable-pmc", "--enable-probe-kernel"] if python else ["--pmc", "--probe"])
    mcores, rss = _measure(flags, python=python)
    print(f"\non-device: {mcores:.1f} millicores, {rss:.1f} MiB (request {cpu_req}m, limit {mem_lim} MiB)")
    assert mcores < cpu_req  # the PMC helper's polling runtime thread is frozen between reads
    assert rss < mem_lim
