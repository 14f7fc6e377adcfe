"""The DaemonSet's security contexts against what a full-capability root exporter reads (ADVICE r3,
r4). The base pod keeps SYS_PTRACE and SYS_NICE (deploy/k8s/gpumon-daemonset.yaml); the opt-in
overlays/fdscan/ adds DAC_READ_SEARCH (kept out of the base since round 5: with RuntimeDefault
seccomp it unlocks open_by_handle_at). Here as root with setpriv: the exporter runs with the bounding
set reduced to the base set, the fdscan set and a set without SYS_PTRACE, against a tenant process
owned by another uid:

* the /proc/<pid>/fd scan that checks a process holds /dev/kfd and finds its DRM fds (sysfs fast
  path) needs DAC_READ_SEARCH to list another uid's fd directory and SYS_PTRACE to read its links
  and /proc/<pid>/fdinfo;
* SCHED_FIFO for the sampler (rt_priority) and the HTTP loops (http_rt_priority) needs SYS_NICE;
* the same --once exposition (family and sample counts) comes out as from full root.

The GPU boxes run commands as an ordinary user, so this check lives on the CPU side."""

import json
import os
import shutil
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(os.geteuid() != 0 or not shutil.which("setpriv"), reason="needs root + setpriv")

SCRIPT = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
from gpumon import core
from gpumon.export import promtext
pid = int(sys.argv[2])
# the real amdsmi backend (over the fake library: no GPU here) keeps the /dev/kfd fd check on
ex = core().Exporter({"backend": "amdsmi", "amdsmi_lib": sys.argv[1] + "/libfake_amd_smi.so", "fast_path": False,
                      "listen_addr": "127.0.0.1", "port": 0, "interval_s": 0.05,
                      "rt_priority": 1, "http_rt_priority": 1, "host": "n", "log_level": "error"})
assert ex.start() == ""
ex.wait_for_seq(3, 10)
st = ex.self_stats()
fam = promtext.parse(ex.metrics_text())
r = ex.resolve_pid(pid)
ex.stop()
import os
def probe(f):
    try:
        return f()
    except OSError as e:
        return type(e).__name__
# the reads behind the /dev/kfd check (attribution.cpp holds_kfd) and the fast path's per-process
# engine time (sysfs_fast.cpp: /proc/<pid>/fdinfo) on the tenant's fd 3
fd_dir = probe(lambda: "3" in os.listdir(f"/proc/{pid}/fd"))
fd_link = probe(lambda: os.readlink(f"/proc/{pid}/fd/3"))
fdinfo = probe(lambda: "pos:" in open(f"/proc/{pid}/fdinfo/3").read())
from gpumon import doctor
doc = doctor.fd_table_check(pid=pid)
print(json.dumps({"rt_threads": st["rt_threads"], "http_rt_loops": st["http_rt_loops"],
                  "fd_dir": fd_dir, "fd_link": fd_link, "fdinfo": fdinfo, "doctor": list(doc),
                  "families": len(fam), "samples": sum(len(f["samples"]) for n, f in fam.items()
                                                       if not n.startswith(("gpumon_", "process_")))}))
"""


def _run(bounding, pkg_root):
    tenant = subprocess.Popen(["setpriv", "--reuid", "65534", "--regid", "65534", "--clear-groups", "sh", "-c",
                               "exec 3</etc/hostname; exec sleep 30"])
    time.sleep(0.3)
    try:
        cmd = [sys.executable, "-c", SCRIPT, pkg_root, str(tenant.pid)]
        if bounding is not None:
            cmd = ["setpriv", "--bounding-set", bounding, "--inh-caps", "-all", "--"] + cmd
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        tenant.kill()
        tenant.wait()


def test_daemonset_capability_set_reads_what_root_reads(tmp_path):
    # the package from a directory the capability-reduced root can read (no DAC_OVERRIDE: a home
    # directory owned by another uid is closed to it)
    pkg = tmp_path / "pkg"
    from conftest import make_locked

    make_locked("fakes")
    shutil.copytree(os.path.join(ROOT, "gpumon"), pkg / "gpumon", ignore=shutil.ignore_patterns("__pycache__"))
    shutil.copy(os.path.join(ROOT, "build", "fakes", "libfake_amd_smi.so"), pkg)
    os.chmod(tmp_path, 0o755)
    full = _run(None, str(pkg))
    r3_set = _run("-all,+sys_ptrace,+sys_nice", str(pkg))  # the base DaemonSet's set (and round 3's)
    ds = _run("-all,+sys_ptrace,+sys_nice,+dac_read_search", str(pkg))  # overlays/fdscan/
    no_ptrace = _run("-all,+sys_nice,+dac_read_search", str(pkg))
    print("\nfull root:", full, "\nround-3 set:", r3_set, "\nDaemonSet set:", ds, "\nwithout SYS_PTRACE:", no_ptrace)
    ok = {"fd_dir": True, "fd_link": "/etc/hostname", "fdinfo": True}
    assert {k: full[k] for k in ok} == ok
    # the base set (SYS_PTRACE + SYS_NICE) cannot list another uid's fd table: the directory is
    # mode 0500 of the tenant's uid, so a root without DAC_READ_SEARCH is refused (the overlay's job)
    assert r3_set["fd_dir"] == "PermissionError"
    # the fdscan overlay's set (+ DAC_READ_SEARCH) reads all three, as full root does
    assert {k: ds[k] for k in ok} == ok
    # ... and the fd links / fdinfo still need SYS_PTRACE on top (ptrace_may_access)
    assert no_ptrace["fd_dir"] is True and no_ptrace["fd_link"] == "PermissionError"
    # `gpumon doctor` names the missing capability in each case
    assert full["doctor"][0] == ds["doctor"][0] == "ok"
    assert r3_set["doctor"][0] == "warn" and "CAP_DAC_READ_SEARCH" in r3_set["doctor"][1]
    assert no_ptrace["doctor"][0] == "warn" and "CAP_SYS_PTRACE" in no_ptrace["doctor"][1]
    # SCHED_FIFO sampler + device workers and both HTTP loops under SYS_NICE
    assert ds["rt_threads"] == full["rt_threads"] > 0 and ds["http_rt_loops"] == full["http_rt_loops"] == 2
    assert (ds["families"], ds["samples"]) == (full["families"], full["samples"])
