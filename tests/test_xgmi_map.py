"""xGMI peer identity from one source (csrc/core/xgmi_map.cpp): amdsmi_get_link_metrics
entries carry the peer BDF AND their own read/write KB; the exporter pairs each entry with the
gpu_metrics slot whose accumulators it matches, instead of trusting that entry k describes slot k.
The reference never queried NVLink (/root/reference/gpu.py:104-116); SURVEY D7 names these fields.

The mock lists one entry per slot; `link_order=reverse|rotate` scrambles the entry order and
`link_offset=1` gives the entries' counters another origin (only per-interval deltas can pair them).
"""

import time

from gpumon.export import promtext

N_LINKS = 7


def _peer_of_slot(ex, dev):
    fam = promtext.parse(ex.metrics_text())
    return {int(l["link"]): l["peer_bdf"] for _, l, v in fam["gpu_xgmi_link_up"]["samples"] if l["gpu_id"] == str(dev)}


def _truth(dev, gpus):
    # the mock's physical wiring: slot k of device dev leads to device (dev + k) % (gpus + 1)
    return {k: "0000:%02x:00.0" % (0x05 + 0x20 * ((dev + k) % max(2, gpus + 1))) for k in range(1, N_LINKS + 1)}


def _distinct_traffic(ex, dev):
    for k in range(1, N_LINKS + 1):
        ex.mock_set_xgmi(dev, k, 5.0 * k)  # GB/s: every link distinguishable


def _self_metric(ex, name, dev):
    return promtext.one(promtext.parse(ex.metrics_text()), name, gpu_id=str(dev))


def test_positional_order_is_verified_not_assumed(mock_exporter):
    ex = mock_exporter(backend="mock:gpus=2,mode=load", link_every=2, sample_threads=0)
    _distinct_traffic(ex, 0)
    for _ in range(3):
        ex.tick()
        time.sleep(0.02)
    assert _peer_of_slot(ex, 0) == _truth(0, 2)
    assert _self_metric(ex, "gpumon_xgmi_slot_map_verified", 0) == N_LINKS
    assert _self_metric(ex, "gpumon_xgmi_slot_map_mismatch", 0) == 0
    assert _self_metric(ex, "gpumon_xgmi_slot_map_unverified", 0) == 0


def test_permuted_entries_paired_by_absolute_counters(mock_exporter):
    """A library listing the entries in another order than the table's slots: the first refresh
    already pairs them (both sources' counters agree at the same instant), so every slot's rate is
    exported under its real peer."""
    for order in ("reverse", "rotate"):
        ex = mock_exporter(backend=f"mock:gpus=2,mode=load,link_order={order}", link_every=1, sample_threads=0)
        _distinct_traffic(ex, 0)
        ex.tick()
        time.sleep(0.05)
        ex.tick()
        assert _peer_of_slot(ex, 0) == _truth(0, 2), order
        assert _self_metric(ex, "gpumon_xgmi_slot_map_mismatch", 0) > 0, order
        # the traffic follows the peer: slot k carries 5k GB/s, and so does its peer label
        fam = promtext.parse(ex.metrics_text())
        for k in range(1, N_LINKS + 1):
            rate = promtext.one(fam, "gpu_xgmi_read_bytes_per_second", gpu_id="0", link=str(k))
            assert abs(rate / 1e9 - 5.0 * k) < 0.5 * k, (order, k, rate)


def test_permuted_entries_with_another_counter_origin_paired_by_deltas(mock_exporter):
    """Entry counters that never equal the table's (another origin): the pairing comes from the
    per-interval deltas of two refreshes; until then the peers are positional and counted as
    unverified."""
    ex = mock_exporter(backend="mock:gpus=2,mode=load,link_order=reverse,link_offset=1", link_every=1,
                       sample_threads=0)
    ex.tick()  # every link carries the same traffic so far: nothing to go on
    assert _self_metric(ex, "gpumon_xgmi_slot_map_unverified", 0) == N_LINKS
    _distinct_traffic(ex, 0)
    ex.tick()
    time.sleep(0.2)  # >= 64 MB per link between refreshes
    ex.tick()
    assert _peer_of_slot(ex, 0) == _truth(0, 2)
    assert _self_metric(ex, "gpumon_xgmi_slot_map_verified", 0) == N_LINKS


def test_balanced_traffic_cannot_pair_and_says_so(mock_exporter):
    """Every link carrying the same bytes (a ring all-reduce, or idle) cannot tell entries apart:
    nothing is verified, and a scrambled order is not silently 'confirmed'."""
    ex = mock_exporter(backend="mock:gpus=2,mode=load,link_order=rotate", link_every=1, sample_threads=0)
    for _ in range(3):
        ex.tick()
        time.sleep(0.05)
    assert _self_metric(ex, "gpumon_xgmi_slot_map_verified", 0) == 0
    assert _self_metric(ex, "gpumon_xgmi_slot_map_unverified", 0) == N_LINKS


def test_pairing_survives_traffic_going_idle(mock_exporter):
    """Once paired, an entry keeps its slot while later refreshes carry no evidence."""
    ex = mock_exporter(backend="mock:gpus=2,mode=idle,link_order=reverse", link_every=1, sample_threads=0)
    _distinct_traffic(ex, 0)
    ex.tick()
    time.sleep(0.05)
    ex.tick()
    assert _peer_of_slot(ex, 0) == _truth(0, 2)
    for k in range(1, N_LINKS + 1):
        ex.mock_set_xgmi(0, k, 0.0)
    for _ in range(3):
        ex.tick()
        time.sleep(0.02)
    assert _peer_of_slot(ex, 0) == _truth(0, 2)


def test_failed_link_refresh_keeps_peer_labels(mock_exporter):
    """a link-refresh tick whose device sample timed out (or whose link-metrics read
    failed) used to count as refreshed, so the next link_every ticks copied an empty identity.
    Now the last identity is carried and the refresh is retried on the next tick."""
    ex = mock_exporter(backend="mock:gpus=1,mode=load", link_every=3, device_timeout_s=0.1)
    ex.tick()  # refresh (tick 0)
    want = _peer_of_slot(ex, 0)
    assert want and all(want.values())
    ex.tick()
    ex.tick()
    ex.mock_set_hang_ms(400.0, 0)  # tick 3 is a refresh tick: the device times out
    ex.tick()
    ex.mock_set_hang_ms(0.0, 0)
    time.sleep(0.5)  # the hung call returns
    calls = ex.mock_link_calls(0)
    for _ in range(2):
        ex.tick()
        assert _peer_of_slot(ex, 0) == want
    assert ex.mock_link_calls(0) == calls + 1  # the failed refresh was retried once, not every tick
    ex.mock_set_link_fail(0, True)  # the link-metrics call itself fails on the next refresh
    for _ in range(4):
        ex.tick()
        assert _peer_of_slot(ex, 0) == want
    ex.mock_set_link_fail(0, False)
    ex.tick()
    assert _peer_of_slot(ex, 0) == want


def test_real_backend_pairs_a_permuted_library_order(core, monkeypatch):
    """The real AmdSmiBackend against the fake libamd_smi whose link-metrics entries describe the
    table's slots in a scrambled order (FAKE_AMDSMI_LINK_SLOTS): every slot's bytes still go out
    under the peer BDF of the entry that matches its counters (bus 0x40 + slot in the fake)."""
    from conftest import make_locked
    from test_amdsmi_fake import FAKE

    make_locked("fakes")
    for slots in ("0,1,2,3,4,5,6", "7,6,5,4,3,2,1", "3,0,7,1,6,2,5,4"):
        monkeypatch.setenv("FAKE_AMDSMI_GPUS", "1")
        monkeypatch.setenv("FAKE_AMDSMI_LINK_SLOTS", slots)
        ex = core.Exporter({"backend": "amdsmi", "amdsmi_lib": FAKE, "serve_http": False, "interval_s": 0,
                            "host": "n1", "verify_kfd": False, "init_retry_s": 0.0, "link_every": 1})
        assert ex.start() == ""
        try:
            ex.tick()
            ex.tick()
            peers = _peer_of_slot(ex, 0)
            listed = [int(x) for x in slots.split(",") if int(x) > 0]
            for k in listed:
                assert peers[k] == "0000:%02x:00.0" % (0x40 + k), (slots, k, peers)
            positional = all(int(x) == j for j, x in enumerate(slots.split(",")))
            assert (_self_metric(ex, "gpumon_xgmi_slot_map_mismatch", 0) == 0) == positional, slots
            assert _self_metric(ex, "gpumon_xgmi_slot_map_verified", 0) == len(listed)
        finally:
            ex.stop()


# ------------------------------------------------------------- the pairing itself (XgmiSlotMap)
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


def _entries(perm, rd, wr):
    # entry j describes table slot perm[j] (0 = self: no peer, no counters)
    return [{"bdf": "" if k == 0 else "0000:%02x:00.0" % (0x40 + k), "read": rd[k] if k else 0,
             "write": wr[k] if k else 0} for k in perm]


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(perm=st.permutations(list(range(8))),
       rd=st.lists(st.integers(0, 10**12), min_size=8, max_size=8),
       wr=st.lists(st.integers(0, 10**12), min_size=8, max_size=8))
def test_pairing_is_never_wrong_and_never_doubles_a_slot(core, perm, rd, wr):
    _check_pairing(core, perm, rd, wr)


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(perm=st.permutations(list(range(8))),
       rd=st.lists(st.sampled_from([0, 10**9, 2 * 10**9]), min_size=8, max_size=8),
       wr=st.lists(st.sampled_from([0, 10**9]), min_size=8, max_size=8))
def test_pairing_with_many_identical_counters(core, perm, rd, wr):
    """Idle or evenly loaded links (many slots with the same counters): ambiguous entries stay
    unpaired; the ones that are unique still pair right."""
    _check_pairing(core, perm, rd, wr)


def _check_pairing(core, perm, rd, wr):
    """Any entry order, any counters: a paired entry sits on the slot it describes; no slot carries
    two entries; an entry whose counters match exactly one slot's is paired."""
    status = [-1] + [1] * 7
    m = core.XgmiSlotMap()
    slots = m.update(_entries(perm, rd, wr), rd, wr, status)
    used = [s for s in slots if s >= 0]
    assert len(used) == len(set(used))
    for j, k in enumerate(perm):
        if k == 0:
            continue
        same = [q for q in range(1, 8) if abs(rd[q] - rd[k]) <= 65536 + max(rd[q], rd[k]) // 10000
                and abs(wr[q] - wr[k]) <= 65536 + max(wr[q], wr[k]) // 10000]
        exact = [q for q in range(1, 8) if rd[q] == rd[k] and wr[q] == wr[k]]
        if len(exact) == 1 and rd[k] + wr[k] > 0 or len(same) == 1:
            assert slots[j] == k, (perm, slots)  # identified
        assert slots[j] in (k, -1) or j == slots[j], (perm, slots)  # paired right, withheld, or positional


def test_deltas_pair_when_origins_differ_and_older_pairings_yield_to_newer(core):
    status = [-1] + [1] * 7
    rd0 = [0] + [10**9 * k for k in range(1, 8)]
    wr0 = [0] + [5 * 10**8 * k for k in range(1, 8)]
    perm = [0, 3, 1, 2, 7, 6, 5, 4]
    off = 7 * 10**11  # entry counters with another origin: never equal to the table's

    def ents(rd, wr):
        return [{"bdf": "" if k == 0 else f"p{k}", "read": rd[k] + off if k else 0, "write": wr[k] + off if k else 0}
                for k in perm]

    m = core.XgmiSlotMap()
    assert m.update(ents(rd0, wr0), rd0, wr0, status) == list(range(8))  # nothing to go on: positional
    assert m.verified == 0 and m.unverified == 7
    rd1 = [r + 10**6 * (3 * k + 1) for k, r in enumerate(rd0)]  # distinct traffic per link (KB)
    wr1 = [w + 10**6 * (2 * k + 5) for k, w in enumerate(wr0)]
    slots = m.update(ents(rd1, wr1), rd1, wr1, status)
    assert slots[1:] == perm[1:] and m.verified == 7 and m.mismatched == 7  # none sits at its position
    # idle afterwards: the pairing holds
    assert m.update(ents(rd1, wr1), rd1, wr1, status)[1:] == perm[1:]
