"""The amdsmi backend's sysfs/KFD fast path (csrc/core/sysfs_fast.*) on CPU.

A fake sysfs tree holds a gpu_metrics v1.8 blob packed here with `struct` from the kernel layout
(an encoding independent of the C++ struct), mem_info_* files and KFD proc entries; the fake
libamd_smi supplies enumeration. Checks: the fast path engages only when the decoded table agrees
with libamd_smi on the stable fields, the exported values then come from sysfs, KFD process rows
carry fdinfo gfx time, and a layout/header mismatch falls back to libamd_smi.
"""

import os
import struct

import pytest

from conftest import make_locked
from gpumon.export import promtext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE = os.path.join(ROOT, "build", "fakes", "libfake_amd_smi.so")
NA16, NA32, NA64 = 0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF


def pack_v18(d=0, gfx=77, xgmi_width=16, revision=8, fw_ts=5_000_000_000, n=1):
    """gpu_metrics_v1_8, little endian, natural alignment spelled out as explicit pad bytes."""
    b = struct.pack("<HBB", 3872, 1, revision)
    b += struct.pack("<6H", 46 + d, 33, 43, 600, gfx, 12)
    b += struct.pack("<3Q", 8192, 1_000_000 + n * 1_000_000, n * 1_000_000_000)
    b += struct.pack("<7I", n * 1000, 0, n * 100, 0, 0, 0, 0)
    b += struct.pack("<4H", 16, 320, xgmi_width, 38)
    b += struct.pack("<2I", n * gfx * 1000, n * 12 * 1000)
    b += b"\0" * 4
    b += struct.pack("<5Q", NA64, 18, 0, 0, 0)
    b += struct.pack("<2I", 0, 0)
    b += struct.pack("<8Q", *([0] + [n * 1_000_000 * k for k in range(1, 8)]))
    b += struct.pack("<8Q", *([0] + [n * 500_000 * k for k in range(1, 8)]))
    b += struct.pack("<8H", NA16, 1, 1, 1, 1, 1, 1, 1) + struct.pack("<H", 0)
    b += b"\0" * 6
    b += struct.pack("<Q", fw_ts)
    b += struct.pack("<8H", *[2100 - k for k in range(8)])
    b += struct.pack("<4H", 1200, NA16, NA16, NA16) + struct.pack("<4H", 29, NA16, NA16, NA16)
    b += struct.pack("<4H", 22, NA16, NA16, NA16) + struct.pack("<2H", 2000, 1)
    b += b"\0" * 4
    for x in range(8):
        busy = [gfx] * 8 if x == 0 else [NA32] * 8
        acc = [n * gfx * 1000] * 8 if x == 0 else [NA64] * 8
        b += struct.pack("<8I", *busy) + struct.pack("<40H", *([NA16] * 40)) + struct.pack("<4H", *([NA16] * 4))
        b += struct.pack("<8Q", *acc) + struct.pack("<32Q", *([NA64] * 32))
    b += struct.pack("<I", 0) + b"\0" * 4
    assert len(b) == 3872
    return b


def make_tree(tmp, gpus=2, blob_kw=None, procs=((4242, 0),)):
    sysr, procr = tmp / "sys", tmp / "proc"
    for d in range(gpus):
        dev = sysr / "bus" / "pci" / "devices" / f"0000:{0x26 + 0x20 * d:02x}:00.0"
        dev.mkdir(parents=True)
        (dev / "gpu_metrics").write_bytes(pack_v18(d=d, **(blob_kw or {})))
        (dev / "mem_info_vram_used").write_text(f"{(123 + d) << 20}\n")
        (dev / "mem_info_vram_total").write_text(f"{288 << 30}\n")
        (dev / "mem_info_gtt_used").write_text(f"{7 << 20}\n")
    for pid, d in procs:
        kp = sysr / "class" / "kfd" / "kfd" / "proc" / str(pid)
        (kp / f"stats_{36622 + d}").mkdir(parents=True)
        (kp / f"vram_{36622 + d}").write_text(f"{2 << 30}\n")
        (kp / f"stats_{36622 + d}" / "cu_occupancy").write_text("17\n")
        fd, fdinfo = procr / str(pid) / "fd", procr / str(pid) / "fdinfo"
        fd.mkdir(parents=True, exist_ok=True)
        fdinfo.mkdir(exist_ok=True)
        a, b = str(5 + 10 * d), str(6 + 10 * d)
        os.symlink(f"/dev/dri/renderD{152 + d}", fd / a)
        os.symlink(f"/dev/dri/renderD{152 + d}", fd / b)  # dup() of the same DRM file
        if not (fd / "7").is_symlink():
            os.symlink("/dev/null", fd / "7")
        for n in (a, b):
            (fdinfo / n).write_text("pos:\t0\nflags:\t02100002\ndrm-driver:\tamdgpu\ndrm-client-id:\t7\n"
                                    "drm-engine-gfx:\t5000000 ns\ndrm-memory-vram:\t1048576 KiB\n"
                                    "drm-memory-gtt:\t2048 KiB\n")
    return sysr, procr


@pytest.fixture(scope="module", autouse=True)
def fake_lib():
    make_locked("fakes")


@pytest.fixture
def exporter(core, monkeypatch):
    made = []

    def make(sysr, procr, **over):
        for k in ("FAKE_AMDSMI_GPUS", "FAKE_AMDSMI_CPX", "FAKE_AMDSMI_NO_METRICS"):
            monkeypatch.delenv(k, raising=False)
        cfg = {"backend": "amdsmi", "amdsmi_lib": FAKE, "serve_http": False, "interval_s": 0, "host": "n1",
               "verify_kfd": False, "init_retry_s": 0.0, "sysfs_root": str(sysr), "procfs_root": str(procr)}
        cfg.update(over)
        ex = core.Exporter(cfg)
        assert ex.start() == ""
        made.append(ex)
        return ex

    yield make
    for ex in made:
        ex.stop()


def test_fast_path_engages_and_values_come_from_sysfs(exporter, tmp_path):
    sysr, procr = make_tree(tmp_path)
    ex = exporter(sysr, procr)
    st = ex.self_stats()
    assert st["fast_path_devices"] == 2 and st["fast_path_status"] == "sysfs"
    ex.tick()
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpumon_fast_path_devices") == 2
    assert promtext.one(fam, "node_gpu_gpu_util", gpu_id="0") == 77  # the blob's value, not amdsmi's 37
    assert promtext.one(fam, "node_gpu_mem_used", gpu_id="1") == 124
    assert promtext.one(fam, "gpu_temperature_celsius", gpu_id="1", sensor="hotspot") == 47
    assert promtext.one(fam, "gpu_gtt_used_bytes", gpu_id="0") == 7 << 20
    assert promtext.values(fam, "gpu_xcd_busy_percent", gpu_id="0") == [77] * 8
    assert promtext.one(fam, "gpu_clock_mhz", gpu_id="0", clock="soc") == 1200


def test_kfd_processes_with_fdinfo(exporter, tmp_path):
    sysr, procr = make_tree(tmp_path)
    ex = exporter(sysr, procr)
    ex.tick()
    rows = [r for r in ex.pod_rows() if not r["idle"]]
    assert [(r["dev"], r["pid"]) for r in rows] == [(0, "4242")]
    r = rows[0]
    assert r["used_memory_bytes"] == 1 << 30  # fdinfo drm-memory-vram (dup'ed fd counted once)
    assert r["cu_occupancy"] == 17
    fam = promtext.parse(ex.metrics_text())
    assert promtext.one(fam, "gpu_process_count", gpu_id="0") == 1
    assert promtext.one(fam, "gpu_process_count", gpu_id="1") == 0


def test_layout_mismatch_falls_back_to_amdsmi(exporter, tmp_path):
    sysr, procr = make_tree(tmp_path, blob_kw={"xgmi_width": 8})
    ex = exporter(sysr, procr)
    st = ex.self_stats()
    assert st["fast_path_devices"] == 0
    assert "xgmi_link_width" in st["fast_path_status"]
    ex.tick()
    assert promtext.one(promtext.parse(ex.metrics_text()), "node_gpu_gpu_util", gpu_id="0") == 37


def test_unknown_table_revision_rejected(exporter, tmp_path):
    sysr, procr = make_tree(tmp_path, blob_kw={"revision": 9})
    ex = exporter(sysr, procr)
    assert ex.self_stats()["fast_path_devices"] == 0


def test_fast_path_can_be_disabled(exporter, tmp_path):
    sysr, procr = make_tree(tmp_path)
    ex = exporter(sysr, procr, fast_path=False)
    assert ex.self_stats()["fast_path_devices"] == 0
    ex.tick()
    assert promtext.one(promtext.parse(ex.metrics_text()), "node_gpu_gpu_util", gpu_id="0") == 37


def test_compare_tables_binding(core, tmp_path, monkeypatch):
    monkeypatch.delenv("FAKE_AMDSMI_GPUS", raising=False)
    sysr, _ = make_tree(tmp_path)
    r = core.amdsmi_compare_tables(FAKE, str(sysr), 1)
    assert r["error"] == ""
    rows = {name: (a, s) for name, a, s in r["rows"]}
    assert rows["temperature_hotspot"] == (47, 47)
    assert rows["average_gfx_activity"] == (37, 77)
    assert rows["xgmi_link_status[3]"] == (1, 1)


def test_fd_tables_are_shared_across_gpus_and_refreshed_off_tick(exporter, tmp_path, core):
    """A process on both GPUs has its /proc/<pid>/fd table scanned once per node, not once per
    GPU; a vanished fd makes the next tick's upkeep (after the publish) rescan it, and the tick
    after that reads the new fd."""
    sysr, procr = make_tree(tmp_path, procs=((4242, 0), (4242, 1)))
    core.fd_table_clear()  # the cache is node-wide: an earlier test's due rescans would count here
    pdir = str(procr / "4242")  # counted per entry: scans of other processes' tables do not count here

    def scans():
        return core.fd_table_scans_of(pdir)

    ex = exporter(sysr, procr, sample_threads=2, interval_s=0)  # start() runs the first tick
    ex.tick()
    rows = sorted((r["dev"], r["used_memory_bytes"]) for r in ex.pod_rows() if not r["idle"])
    assert rows == [(0, 1 << 30), (1, 1 << 30)]
    assert scans() == 1  # one scan served both GPUs
    ex.tick()
    assert scans() == 1  # cached
    # the process closes fd 5 and opens fd 9 on GPU 0's render node
    fd, fdinfo = procr / "4242" / "fd", procr / "4242" / "fdinfo"
    text = (fdinfo / "5").read_text().replace("1048576 KiB", "2097152 KiB")
    (fd / "5").unlink()
    (fdinfo / "5").unlink()
    (fd / "6").unlink()
    (fdinfo / "6").unlink()
    os.symlink("/dev/dri/renderD152", fd / "9")
    (fdinfo / "9").write_text(text)
    ex.tick()  # fdinfo/5 is gone: invalidated, rescanned by a worker after this tick's publish
    import time

    deadline = time.time() + 5
    while scans() < 2 and time.time() < deadline:
        time.sleep(0.01)
    # both GPUs' workers lost an fd (5 on GPU 0, 6 on GPU 1): one rescan, or two when the second
    # worker's invalidation lands after the first rescan finished (a loaded host)
    assert 2 <= scans() <= 3
    ex.tick()  # the worker finished its upkeep before taking this tick
    rows = dict((r["dev"], r["used_memory_bytes"]) for r in ex.pod_rows() if not r["idle"])
    assert rows[0] == 2 << 30


def test_reused_pid_is_not_read_at_the_old_fd_numbers(exporter, tmp_path, core):
    """the node-wide fd-table cache was keyed by /proc/<pid> only and kept an entry 60 s
    after last use, so a pid reused within that time was read at the old process's fd numbers
    until a read failed or the 10 s refresh. An entry now goes as soon as its pid leaves the KFD
    process list; the new process is scanned afresh."""
    import shutil

    sysr, procr = make_tree(tmp_path, gpus=1)
    core.fd_table_clear()
    ex = exporter(sysr, procr, sample_threads=0)
    ex.tick()
    row = next(r for r in ex.pod_rows() if r["pid"] == "4242")
    assert row["used_memory_bytes"] == 1 << 30  # fdinfo VRAM (fds 5, 6)
    # the process exits: gone from KFD and /proc
    kp = sysr / "class" / "kfd" / "kfd" / "proc" / "4242"
    shutil.rmtree(kp)
    shutil.rmtree(procr / "4242")
    ex.tick()
    assert not [r for r in ex.pod_rows() if r["pid"] == "4242"]
    assert core.fd_table_stats()["entries"] == 0  # dropped with the pid, not kept for 60 s
    # a new process gets pid 4242 again, with its DRM file at another fd number
    (kp / "stats_36622").mkdir(parents=True)
    (kp / "vram_36622").write_text(f"{2 << 30}\n")
    (kp / "stats_36622" / "cu_occupancy").write_text("0\n")
    fd, fdinfo = procr / "4242" / "fd", procr / "4242" / "fdinfo"
    fd.mkdir(parents=True)
    fdinfo.mkdir()
    os.symlink("/dev/dri/renderD152", fd / "11")
    (fdinfo / "11").write_text("drm-driver:\tamdgpu\ndrm-client-id:\t9\ndrm-engine-gfx:\t1 ns\n"
                               "drm-memory-vram:\t3145728 KiB\n")
    ex.tick()
    row = next(r for r in ex.pod_rows() if r["pid"] == "4242")
    assert row["used_memory_bytes"] == 3 << 30, row  # the new process's fd 11, not the old fds


def _kfd_proc(sysr, pid, d=0, occ=17):
    kp = sysr / "class" / "kfd" / "kfd" / "proc" / str(pid)
    (kp / f"stats_{36622 + d}").mkdir(parents=True)
    (kp / f"vram_{36622 + d}").write_text(f"{1 << 30}\n")
    (kp / f"stats_{36622 + d}" / "cu_occupancy").write_text(f"{occ}\n")
    return kp


def test_between_tick_kfd_scans_read_arrivals_and_retry_after_a_failed_listing(exporter, tmp_path):
    """The device workers' between-tick cu_occupancy reads through the sysfs fast path (the path a
    real node runs; tests/test_occupancy.py drives the same worker logic through the mock backend).
    A process that appears between ticks is found by the worker's own KFD listing and read from
    then on; a listing that fails (the KFD proc dir gone) is counted and retried, not latched off."""
    import shutil
    import time

    sysr, procr = make_tree(tmp_path, gpus=1)
    ex = exporter(sysr, procr, interval_s=0.3, occ_samples=10, sample_threads=-1)
    assert ex.wait_for_seq(ex.seq + 2, 10)
    row = next(r for r in ex.pod_rows() if r["pid"] == "4242")
    assert row["occ_samples"] >= 4, row  # sub-samples between ticks + the tick's own read
    assert row["cu_occupancy"] == 17
    # a tenant arrives right after a tick; no /proc entry (a pid of another namespace)
    s0 = ex.seq
    assert ex.wait_for_seq(s0 + 1, 10)
    _kfd_proc(sysr, 5151, occ=200)
    deadline = time.time() + 10
    first = None
    while first is None and time.time() < deadline:
        assert ex.wait_for_seq(ex.seq + 1, 10)
        first = next((r for r in ex.pod_rows() if r["pid"] == "5151"), None)
    assert first is not None
    # the first tick that lists it already carries reads from before the tick
    assert first["occ_samples"] >= 2, first
    assert first["cu_occupancy"] == 200 and first["proc_gfx_util"] == 100
    assert ex.self_stats()["occupancy_reads"] > 0
    assert ex.self_stats()["occupancy_scan_failures"] == 0
    # the KFD proc directory disappears: each listing fails and is retried with a backoff
    shutil.rmtree(sysr / "class" / "kfd" / "kfd" / "proc")
    deadline = time.time() + 10
    while ex.self_stats()["occupancy_scan_failures"] == 0 and time.time() < deadline:
        time.sleep(0.05)
    assert ex.self_stats()["occupancy_scan_failures"] >= 1
    # and it comes back: the retry (1 s backoff) lists the new tenant again
    _kfd_proc(sysr, 6161, occ=50)
    deadline = time.time() + 10
    row = None
    while row is None and time.time() < deadline:
        assert ex.wait_for_seq(ex.seq + 1, 10)
        row = next((r for r in ex.pod_rows() if r["pid"] == "6161"), None)
    assert row is not None and row["cu_occupancy"] == 50


def test_process_of_another_gpu_is_not_reasked_every_tick_but_is_picked_up_later(exporter, tmp_path):
    """The KFD proc dir lists the host's processes on every GPU. A process found not to be on a
    GPU is not asked again by that GPU for a second (an open() that fails, per process per tick and
    per scan); when it starts using the GPU it shows up within that second."""
    import time

    sysr, procr = make_tree(tmp_path, gpus=2, procs=((4242, 0),))
    ex = exporter(sysr, procr, sample_threads=0)
    ex.tick()
    rows = sorted((r["dev"], r["pid"]) for r in ex.pod_rows() if not r["idle"])
    assert rows == [(0, "4242")]
    # the process opens GPU 1 too
    kp = sysr / "class" / "kfd" / "kfd" / "proc" / "4242"
    (kp / "stats_36623").mkdir()
    (kp / "vram_36623").write_text(f"{1 << 30}\n")
    (kp / "stats_36623" / "cu_occupancy").write_text("5\n")
    ex.tick()
    assert sorted((r["dev"], r["pid"]) for r in ex.pod_rows() if not r["idle"]) == [(0, "4242")]  # cached
    time.sleep(1.1)
    ex.tick()
    assert sorted((r["dev"], r["pid"]) for r in ex.pod_rows() if not r["idle"]) == [(0, "4242"), (1, "4242")]


def test_kfd_per_pid_files_are_kept_open_and_closed_when_the_process_leaves(exporter, tmp_path):
    """The per-pid KFD files (vram_<gpu>, stats_<gpu>/cu_occupancy) are opened once and re-read
    with pread(0): the 20 sub-samples per tick each cost one read instead of open + read + close.
    A value written between ticks is what the next read returns (same inode, re-read from 0). The
    files of a process that left the KFD listing are closed at the next process list."""
    import shutil

    sysr, procr = make_tree(tmp_path, gpus=1)
    ex = exporter(sysr, procr, sample_threads=0)
    for _ in range(3):
        ex.tick()
    st = ex.self_stats()
    assert st["kfd_files_open"] == 2  # vram + cu_occupancy of pid 4242 on GPU 0
    assert st["kfd_reads_cached"] >= 4
    occ = sysr / "class" / "kfd" / "kfd" / "proc" / "4242" / "stats_36622" / "cu_occupancy"
    occ.write_text("211\n")
    ex.tick()
    assert next(r for r in ex.pod_rows() if r["pid"] == "4242")["cu_occupancy"] == 211
    shutil.rmtree(sysr / "class" / "kfd" / "kfd" / "proc" / "4242")  # the process exited
    ex.tick()
    assert ex.self_stats()["kfd_files_open"] == 0
    assert not [r for r in ex.pod_rows() if not r["idle"] and r["dev"] == 0]


def _queues(kp, gpu_ids):
    """KFD's per-process queue list: one proc/<pid>/queues/<qid>/gpuid per hardware queue."""
    for q, gid in enumerate(gpu_ids):
        (kp / "queues" / str(q)).mkdir(parents=True)
        (kp / "queues" / str(q) / "gpuid").write_text(f"{gid}\n")
        (kp / "queues" / str(q) / "type").write_text("0\n")
    (kp / "queues").mkdir(exist_ok=True)


def test_kfd_queue_list_classifies_peer_contexts(exporter, tmp_path, core):
    """the sysfs fast path reads proc/<pid>/queues/*/gpuid. Rank 7070 computes on GPU 0
    (2 queues there) and holds a 2 GiB context on GPU 1 with no queue and no waves: a peer context
    whatever its VRAM (the 512 MiB threshold alone kept it). Process 8080 holds 64 MiB on GPU 1
    with a queue there but no wave this tick, and its main work on GPU 0: it keeps both rows."""
    sysr, procr = make_tree(tmp_path, gpus=2, procs=())
    a0, a1 = _kfd_proc(sysr, 7070, d=0, occ=120), None
    (a0 / "stats_36623").mkdir()
    (a0 / "vram_36623").write_text(f"{2 << 30}\n")
    (a0 / "stats_36623" / "cu_occupancy").write_text("0\n")
    _queues(a0, [36622, 36622])
    b = _kfd_proc(sysr, 8080, d=0, occ=90)
    (b / "stats_36623").mkdir()
    (b / "vram_36623").write_text(f"{64 << 20}\n")
    (b / "stats_36623" / "cu_occupancy").write_text("0\n")
    _queues(b, [36622, 36623])
    ex = exporter(sysr, procr, sample_threads=0)
    for _ in range(2):
        ex.tick()
    rows = sorted((r["dev"], r["pid"]) for r in ex.pod_rows() if not r["idle"])
    assert rows == [(0, "7070"), (0, "8080"), (1, "8080")], rows
    assert ex.self_stats()["hidden_peer_contexts"] == 1
    # without the queue list (an unreadable directory) the VRAM threshold decides again: 7070's
    # 2 GiB context on GPU 1 is then a workload row, 8080's 64 MiB one a peer context
    import shutil

    for pid in (7070, 8080):
        shutil.rmtree(sysr / "class" / "kfd" / "kfd" / "proc" / str(pid) / "queues")
    core.kfd_queue_tables_clear()  # the node-wide lists are otherwise reread only after 2 s
    ex2 = exporter(sysr, procr, sample_threads=0)
    for _ in range(2):
        ex2.tick()
    rows = sorted((r["dev"], r["pid"]) for r in ex2.pod_rows() if not r["idle"])
    assert rows == [(0, "7070"), (0, "8080"), (1, "7070")], rows


def test_kfd_queue_list_is_scanned_once_for_every_gpu(exporter, tmp_path, core):
    """One process's queue directory names the GPU of each queue, so the node-wide table reads it
    once per rescan period for all device workers (8 GPUs: 8x fewer scans); each GPU still gets its
    own count, and a process that left the KFD listing is dropped from the table."""
    import shutil

    sysr, procr = make_tree(tmp_path, gpus=2, procs=())
    kp = _kfd_proc(sysr, 9090, d=0, occ=50)
    (kp / "stats_36623").mkdir()
    (kp / "vram_36623").write_text(f"{1 << 30}\n")
    (kp / "stats_36623" / "cu_occupancy").write_text("40\n")
    _queues(kp, [36622, 36622, 36622, 36623])
    ex = exporter(sysr, procr, sample_threads=-1)  # one worker per GPU, in parallel
    for _ in range(3):
        ex.tick()
    q = {r["dev"]: r["queues"] for r in ex.pod_rows() if r["pid"] == "9090"}
    assert q == {0: 3, 1: 1}, q
    # 3 ticks x 2 GPUs inside one rescan period: one scan (two if both workers met a stale entry
    # at the same instant)
    assert 1 <= core.kfd_queue_scans(str(sysr), 9090) <= 2
    shutil.rmtree(kp)
    ex.tick()
    assert core.kfd_queue_scans(str(sysr), 9090) == 0  # dropped with the process
