"""xGMI link-map validator (gpumon/parallel/xgmi.py validate_pair, `gpumon xgmi`) on the mock
backend: the link whose counter moves under a peer copy must be the one the exporter maps to the
destination GPU's BDF. On hardware the copier is a torch peer copy (hipMemcpyPeerAsync)."""

import time

from gpumon.parallel.xgmi import busiest_link, validate_pair


class _FakeCopier:
    def __init__(self, src, dst):
        self.src, self.dst = src, dst

    def run(self, seconds):
        time.sleep(seconds)
        return 50e9


def test_busiest_link():
    assert busiest_link({"xgmi_wr_Bps": [0, 1e9, 5e9, 2e9]}) == (2, 5e9)
    assert busiest_link({}) == (-1, 0.0)


def _exporter(core):
    ex = core.Exporter({"backend": "mock:gpus=8,mode=idle", "serve_http": False, "interval_s": 0.05,
                        "link_every": 1})
    ex.start()
    return ex


def test_validate_pair_finds_the_peer_link(core):
    ex = _exporter(core)
    try:
        # mock topology: device 0's link k leads to device k. Drive 0 -> 3 over link 3.
        ex.mock_set_xgmi(0, 3, 60.0)
        ex.mock_set_xgmi(3, 5, 60.0)  # on the receiver the traffic arrives on its own link 5
        r = validate_pair(ex, 0, 3, copier_factory=_FakeCopier, seconds=0.5, interval=0.05)
    finally:
        ex.stop()
    assert r["src_link"] == 3 and r["src_link_tx_GBps"] > 20
    assert r["dst_link"] == 5
    assert r["src_link_peer_bdf"] == r["dst_bdf"] == "0000:65:00.0"
    assert r["peer_matches"] and r["copy_GBps"] == 50.0


def test_validate_pair_flags_a_wrong_map(core):
    ex = _exporter(core)
    try:
        ex.mock_set_xgmi(0, 2, 60.0)  # traffic shows up on link 2 (peer = device 2), copy went to 3
        r = validate_pair(ex, 0, 3, copier_factory=_FakeCopier, seconds=0.4, interval=0.05)
    finally:
        ex.stop()
    assert r["src_link"] == 2 and not r["peer_matches"]


def test_cli_skips_on_single_gpu(capsys):
    from gpumon.cli import main

    assert main(["xgmi"]) == 0
    assert "skipped" in capsys.readouterr().out
