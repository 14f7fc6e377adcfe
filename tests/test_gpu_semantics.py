"""Metric semantics checked against known work on one MI355X (the PCIe gauge
read 18-35 "GB/s" on idle GPUs for three rounds because no test drove PCIe traffic). Each test puts a
load of known shape on the GPU and checks that the exported value moves the way its unit and HELP
text say: HBM controller activity under the HBM stream, interval power from the energy accumulator
against the firmware's power and the energy counter itself, VRAM used against an allocation of
known size. The reference exported utilisation and memory only (/root/reference/gpu.py:132-146).
"""

import time

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _exporter(core):
    ex = core.Exporter({"backend": "amdsmi", "devices": [0], "serve_http": False, "interval_s": 0.0,
                        "host": "gpu-box"})
    assert ex.start() == ""
    return ex


def _window(ex, seconds=2.0, ticks=4):
    """A baseline tick, then `ticks` ticks spread over `seconds`: per tick (fields, rates)."""
    ex.tick()
    out = []
    for _ in range(ticks):
        time.sleep(seconds / ticks)
        ex.tick()
        out.append((ex.samples()[0]["fields"], ex.rates()[0]))
    return out


def _mean(xs):
    xs = [x for x in xs if x is not None]
    return sum(xs) / len(xs) if xs else None


def test_hbm_activity_tracks_the_hbm_stream(core, torch_gpu):
    """node_gpu_mem_bw_util / gpu_umc_activity_avg_percent: the memory controllers' activity. The
    HBM stream (6.5 TB/s, ~80 % of the 8 TB/s peak) must read far above idle and above the MFMA burn,
    which touches almost no HBM."""
    from gpumon.ops.load import SyntheticLoad

    ex = _exporter(core)
    try:
        got = {}
        for kind in ("idle", "mfma", "hbm"):
            if kind == "idle":
                w = _window(ex)
            else:
                with SyntheticLoad(0, kind, hbm_bytes=1 << 30) as load:
                    time.sleep(0.5)
                    w = _window(ex)
                    st = load.stats()
                if kind == "hbm":
                    assert st["tbps"] > 5.0, st  # the stream really ran at full rate
            got[kind] = (_mean([f["umc_util"] for f, _ in w]), _mean([r["mem_activity_avg_pct"] for _, r in w]))
        print(f"\numc activity inst / interval avg %: {got}")
        idle, mfma, hbm = got["idle"], got["mfma"], got["hbm"]
        assert idle[1] < 10 and hbm[1] > 40, got
        assert hbm[1] > mfma[1] + 20, got
        assert abs(hbm[0] - hbm[1]) < 25, got  # the instantaneous gauge tells the same story
    finally:
        ex.stop()


def test_interval_power_agrees_with_the_firmware_and_the_energy_counter(core, torch_gpu):
    """gpu_power_interval_watts is d(energy accumulator) x resolution / dt. Under a steady bf16 burn
    it must agree with the firmware's socket power (a unit or resolution error would not), and the
    exported energy counter (gpu_energy_joules_total) must advance at the same rate."""
    from gpumon.ops.load import SyntheticLoad

    ex = _exporter(core)
    try:
        idle = _window(ex, seconds=1.0, ticks=2)
        with SyntheticLoad(0, "mfma") as _:
            time.sleep(1.0)
            ex.tick()
            e0, t0 = ex.samples()[0]["fields"]["energy_j"], time.monotonic()
            w = _window(ex, seconds=3.0, ticks=6)
            e1, t1 = ex.samples()[0]["fields"]["energy_j"], time.monotonic()
        p_int = _mean([r["power_from_energy_w"] for _, r in w])
        p_fw = _mean([f["power_cur"] for f, _ in w])
        p_energy = (e1 - e0) / (t1 - t0)
        p_idle = _mean([r["power_from_energy_w"] for _, r in idle])
        print(f"\nburn: interval {p_int:.0f} W, firmware current {p_fw:.0f} W, d(energy)/dt {p_energy:.0f} W; "
              f"idle interval {p_idle:.0f} W")
        assert p_int > 300 and p_int > 1.5 * p_idle, (p_int, p_idle)
        assert abs(p_int / p_fw - 1) < 0.15, (p_int, p_fw)
        assert abs(p_energy / p_int - 1) < 0.15, (p_energy, p_int)
    finally:
        ex.stop()


def test_vram_used_tracks_an_allocation(core, torch_gpu):
    """node_gpu_mem_used (MiB) / gpu_vram_used_bytes: a tenant's 8 GiB allocation moves the device's
    VRAM used by 8 GiB, and back when the tenant exits (the reference's mem_used field, gpu.py:139);
    the tenant's pod_gpu row carries it too (KFD's per-process VRAM)."""
    import subprocess
    import sys

    code = ("import sys, time, torch; x = torch.empty(8 << 30, dtype=torch.uint8, device='cuda:0'); x.fill_(1); "
            "torch.cuda.synchronize(); print('ready', flush=True); sys.stdin.readline()")
    ex = _exporter(core)
    try:
        ex.tick()
        before = ex.samples()[0]["fields"]["vram_used"]
        rows0 = sum(r["used_memory_bytes"] for r in ex.pod_rows() if not r["idle"])
        t = subprocess.Popen([sys.executable, "-c", code], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        try:
            assert t.stdout.readline().strip() == "ready"
            ex.tick()
            during = ex.samples()[0]["fields"]["vram_used"]
            rows1 = sum(r["used_memory_bytes"] for r in ex.pod_rows() if not r["idle"])
        finally:
            t.stdin.write("\n")
            t.stdin.flush()
            t.wait(60)
        deadline = time.monotonic() + 10  # the driver returns the tenant's memory when its KFD process ends
        after = during
        while time.monotonic() < deadline and abs(after - before) >= 256 << 20:
            time.sleep(0.2)
            ex.tick()
            after = ex.samples()[0]["fields"]["vram_used"]
        d = (during - before) / 2 ** 30
        dr = (rows1 - rows0) / 2 ** 30
        print(f"\nVRAM used: {before / 2 ** 30:.2f} -> {during / 2 ** 30:.2f} -> {after / 2 ** 30:.2f} GiB; "
              f"pod rows +{dr:.2f} GiB")
        assert 8.0 <= d < 9.0, d  # the 8 GiB plus the tenant runtime's own buffers (~0.5 GiB, r6_kfd_queues.md)
        assert 8.0 <= dr < 9.0, dr
        assert abs(after - before) < 256 << 20, (before, after)
    finally:
        ex.stop()


def test_clocks_and_temperature_respond_to_load(core, torch_gpu):
    """gpu_clock_mhz{clock="gfx"} and gpu_temperature_celsius{sensor="hotspot"} under the burn: the gfx
    clock runs at a working frequency and the hotspot is no cooler than idle."""
    from gpumon.ops.load import SyntheticLoad

    ex = _exporter(core)
    try:
        idle = _window(ex, seconds=1.0, ticks=2)
        with SyntheticLoad(0, "mfma") as _:
            time.sleep(1.0)
            w = _window(ex, seconds=2.0, ticks=4)
        clk = _mean([f["gfxclk_cur"] for f, _ in w])
        hot, hot_idle = _mean([f["temp_hotspot"] for f, _ in w]), _mean([f["temp_hotspot"] for f, _ in idle])
        print(f"\nburn: gfx clock {clk:.0f} MHz, hotspot {hot:.0f} C (idle {hot_idle:.0f} C)")
        assert 1000 < clk <= 2500, clk
        assert hot >= hot_idle - 1, (hot, hot_idle)
    finally:
        ex.stop()
