"""The on-device helper on a real MI355X: killed under load, it is respawned and the samplers
recover (csrc/core/ondevice.cpp OnDevice::helper_check). The helper owns rocprofiler-sdk device
counting contexts and the HIP probe; the kernel frees the dead process's counters, so the new
helper can program them again."""

import os
import signal
import subprocess
import sys
import time

import pytest

from gpumon.export import promtext

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _helpers():
    out = []
    for p in os.listdir("/proc"):
        if p.isdigit():
            try:
                if open(f"/proc/{p}/comm").read().strip() == "gpumon-ondevice" and \
                        int(open(f"/proc/{p}/stat").read().rsplit(")", 1)[1].split()[1]) == os.getpid():
                    out.append(int(p))
            except (OSError, ValueError, IndexError):
                pass
    return out


def test_killed_helper_is_respawned_and_counts_again():
    from gpumon import core

    load = subprocess.Popen([sys.executable, "-m", "gpumon", "load", "--kind", "mfma", "--seconds", "60"], cwd=ROOT,
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    c = core()
    ex = c.Exporter({"backend": "amdsmi", "devices": [0], "serve_http": False, "interval_s": 0.0,
                     "processes": False, "log_level": "warn"})
    assert ex.start() == ""
    od = c.OnDevice(ex, {"pmc": True, "probe": True, "pmc_every_s": 60.0, "probe_every_s": 60.0,
                         "pmc_mode": "continuous", "ondevice_isolate": True, "helper_retry_s": 0.5})
    od.start()
    try:
        time.sleep(3)  # the load is running
        od.step()
        time.sleep(0.3)
        od.step()
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        before = promtext.one(fam, "gpu_mfma_util_percent", gpu_id="0")
        assert before > 50, before
        (pid,) = _helpers()
        os.kill(pid, signal.SIGKILL)
        od.step()
        ex.tick()
        assert promtext.one(promtext.parse(ex.metrics_text()), "gpumon_pmc_up") == 0
        time.sleep(0.6)
        od.step()  # respawn: PMC init in the new helper, contexts started, probes recreated
        time.sleep(0.3)
        od.step()
        ex.tick()
        fam = promtext.parse(ex.metrics_text())
        assert od.stats()["helper_restarts"] == 1
        assert promtext.one(fam, "gpumon_pmc_up") == 1
        after = promtext.one(fam, "gpu_mfma_util_percent", gpu_id="0")
        assert abs(after - before) < 15, (before, after)
        assert promtext.one(fam, "gpu_probe_latency_seconds", gpu_id="0") > 0
        assert promtext.one(fam, "gpumon_ondevice_helper_restarts_total") == 1
        (pid2,) = _helpers()
        assert pid2 != pid
    finally:
        od.stop()
        ex.stop()
        load.terminate()
        load.wait(60)
    assert _helpers() == []


@pytest.mark.parametrize("isolate", [False, True], ids=["in_process", "helper"])
def test_probe_pairs_devices_by_pci_address(isolate):
    """The K1 probe's runtime (raw HSA by default) reports each HIP ordinal's PCI address, and the
    sampler pairs it with the exporter's device of the same BDF (libamd_smi): on this box the one
    GPU is probed through that pairing, not by hip_id."""
    from gpumon import core

    c = core()
    ex = c.Exporter({"backend": "amdsmi", "serve_http": False, "interval_s": 0.0, "processes": False,
                     "log_level": "warn"})
    assert ex.start() == ""
    od = c.OnDevice(ex, {"probe": True, "probe_every_s": 60.0, "probe_blocks": 512, "ondevice_isolate": isolate})
    od.start()
    try:
        od.step()
        st = od.stats()
        assert st["probe_by_bdf"] is True and st["probe_devices"] == len(ex.statics()) >= 1, st
        assert st["probe_done"] >= 1, st
    finally:
        od.stop()
        ex.stop()
