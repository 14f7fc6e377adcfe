"""HPACK decoder (csrc/core/hpack.cpp) against RFC 7541 Appendix C, and the native gRPC client's
decoded statuses against a real grpcio server (whose C-core encoder uses the dynamic table and
Huffman strings, like the kubelet's and containerd's Go encoders)."""

import os
import tempfile

import grpc
import pytest
from hypothesis import given, settings, strategies as st

H = bytes.fromhex


def test_huffman_rfc_vectors(core):
    vec = {"www.example.com": "f1e3c2e5f23a6ba0ab90f4ff", "no-cache": "a8eb10649cbf",
           "custom-key": "25a849e95ba97d7f", "custom-value": "25a849e95bb8e8b4bf", "302": "6402",
           "private": "aec3771a4b", "Mon, 21 Oct 2013 20:13:21 GMT": "d07abe941054d444a8200595040b8166e082a62d1bff",
           "https://www.example.com": "9d29ad171863c78f0b97c8e9ae82ae43d3", "307": "640eff",
           "gzip": "9bd9ab",
           "foo=ASDJKHQKBZXOQWEOPIUAXQWEOIU; max-age=3600; version=1":
               "94e7821dd7f2e6c7b335dfdfcd5b3960d5af27087f3672c1ab270fb5291f9587316065c003ed4ee5b1063d5007"}
    for s, hx in vec.items():
        assert core.hpack_huffman_encode(s.encode()).hex() == hx
        assert core.hpack_huffman_decode(H(hx)) == s.encode()


@settings(max_examples=300, deadline=None)
@given(st.binary(max_size=64))
def test_huffman_round_trip_every_byte(b):
    from gpumon import core as _c

    c = _c()
    assert c.hpack_huffman_decode(c.hpack_huffman_encode(b)) == b


def test_huffman_rejects_bad_padding(core):
    with pytest.raises(ValueError):
        core.hpack_huffman_decode(H("f1e3c2e5f23a6ba0ab90f4fe"))  # last pad bit 0
    with pytest.raises(ValueError):
        core.hpack_huffman_decode(H("ffffffff"))  # EOS (30 ones) inside the string


def test_rfc_c3_requests_without_huffman(core):
    r = core.hpack_decode([H("828684410f7777772e6578616d706c652e636f6d"),
                           H("828684be58086e6f2d6361636865"),
                           H("828785bf400a637573746f6d2d6b65790c637573746f6d2d76616c7565")])
    assert r[0]["headers"] == [(":method", "GET"), (":scheme", "http"), (":path", "/"),
                               (":authority", "www.example.com")]
    assert r[0]["table_size"] == 57
    assert r[1]["headers"][-1] == ("cache-control", "no-cache") and r[1]["headers"][3] == (":authority", "www.example.com")
    assert r[1]["table_size"] == 110
    assert r[2]["headers"] == [(":method", "GET"), (":scheme", "https"), (":path", "/index.html"),
                               (":authority", "www.example.com"), ("custom-key", "custom-value")]
    assert r[2]["table_size"] == 164 and r[2]["table_entries"] == 3


def test_rfc_c4_requests_with_huffman(core):
    r = core.hpack_decode([H("828684418cf1e3c2e5f23a6ba0ab90f4ff"),
                           H("828684be5886a8eb10649cbf"),
                           H("828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf")])
    assert r[2]["headers"][-1] == ("custom-key", "custom-value") and r[2]["table_size"] == 164


def test_rfc_c6_responses_with_eviction(core):
    """256-byte table: entries evicted as responses arrive (Appendix C.6)."""
    r = core.hpack_decode([
        H("488264025885aec3771a4b6196d07abe941054d444a8200595040b8166e082a62d1bff6e919d29ad171863c78f0b97c8e9ae82ae43d3"),
        H("4883640effc1c0bf"),
        H("88c16196d07abe941054d444a8200595040b8166e084a62d1bffc05a839bd9ab77ad94e7821dd7f2e6c7b335dfdfcd5b3960d5af27087f3672c1ab270fb5291f9587316065c003ed4ee5b1063d5007"),
    ], table_size=256)
    assert r[0]["headers"] == [(":status", "302"), ("cache-control", "private"),
                               ("date", "Mon, 21 Oct 2013 20:13:21 GMT"), ("location", "https://www.example.com")]
    assert r[0]["table_size"] == 222
    assert r[1]["headers"][0] == (":status", "307") and r[1]["table_size"] == 222
    assert r[2]["headers"][-1] == ("set-cookie", "foo=ASDJKHQKBZXOQWEOPIUAXQWEOIU; max-age=3600; version=1")
    assert r[2]["headers"][3] == ("location", "https://www.example.com")
    assert r[2]["table_size"] == 215 and r[2]["table_entries"] == 3


def test_malformed_blocks_are_errors(core):
    for bad in (H("ff"), H("be"), H("41"), H("3fe13f"), H("4085")):  # truncated int, bad index, ...
        with pytest.raises(ValueError):
            core.hpack_decode([bad])
    with pytest.raises(ValueError):
        core.hpack_decode([H("82" "20")])  # size update after a field


# ------------------------------------------------------------------------------------ gRPC status
@pytest.fixture
def kubelet():
    from oracles.attribution.fake_kubelet import FakeKubelet

    d = tempfile.mkdtemp(prefix="gpumon-kl-")
    k = FakeKubelet(podres_socket=os.path.join(d, "kubelet.sock"), cri_socket=os.path.join(d, "cri.sock"))
    k.start()
    yield k
    k.stop()


def test_ok_call_decodes_status_zero(core, kubelet):
    r = core.grpc_call(kubelet.podres_socket, "/v1.PodResourcesLister/List")
    assert r["ok"] and r["code"] == 0 and r["http_status"] == 200, r


@pytest.mark.parametrize("code,name", [(grpc.StatusCode.UNIMPLEMENTED, "UNIMPLEMENTED"),
                                       (grpc.StatusCode.PERMISSION_DENIED, "PERMISSION_DENIED"),
                                       (grpc.StatusCode.UNAVAILABLE, "UNAVAILABLE")])
def test_error_status_and_message_are_decoded(core, kubelet, code, name):
    kubelet.podres_error = (code, "kubelet says 100% no: é")
    r = core.grpc_call(kubelet.podres_socket, "/v1.PodResourcesLister/List")
    assert not r["ok"] and r["code_name"] == name and r["code"] == code.value[0]
    assert r["message"] == "kubelet says 100% no: é"
    assert r["error"].startswith(f"grpc-status {code.value[0]} {name}")
    with pytest.raises(RuntimeError, match=name):
        core.podresources_list(kubelet.podres_socket)


def test_unknown_method_is_unimplemented(core, kubelet):
    r = core.grpc_call(kubelet.podres_socket, "/v9.Nope/List")
    assert not r["ok"] and r["code_name"] == "UNIMPLEMENTED", r


def test_many_calls_reuse_nothing_stale(core, kubelet):
    """Each call is its own connection with its own dynamic table: 50 mixed ok / error calls."""
    for i in range(50):
        kubelet.podres_error = (grpc.StatusCode.PERMISSION_DENIED, f"no {i}") if i % 3 == 0 else None
        r = core.grpc_call(kubelet.podres_socket, "/v1.PodResourcesLister/List")
        assert (r["code"] == 7 and r["message"] == f"no {i}") if i % 3 == 0 else r["ok"], (i, r)


def test_exporter_exports_the_status(core, kubelet):
    kubelet.podres_error = (grpc.StatusCode.PERMISSION_DENIED, "pod-resources socket is root-only")
    ex = core.Exporter({"backend": "mock:gpus=1", "serve_http": False, "interval_s": 0.0,
                        "pod_resources_socket": kubelet.podres_socket, "cri_socket": kubelet.cri_socket})
    ex.start()
    try:
        ex.tick()
        from gpumon.export import promtext

        fam = promtext.parse(ex.metrics_text())
        assert promtext.one(fam, "gpumon_podresources_up") == 0
        assert promtext.one(fam, "gpumon_podresources_grpc_status") == 7
        assert promtext.one(fam, "gpumon_cri_up") == 1 and promtext.one(fam, "gpumon_cri_grpc_status") == 0
    finally:
        ex.stop()


def test_cri_falls_back_to_v1alpha2(core):
    from oracles.attribution.fake_kubelet import FakeKubelet, FakePod

    d = tempfile.mkdtemp(prefix="gpumon-cri-")
    k = FakeKubelet(cri_socket=os.path.join(d, "cri.sock"), cri_api="runtime.v1alpha2")
    k.pods.append(FakePod("p", "ns", "u1", containers={"c": ("cid123", ["0"])}))
    with k:
        cs, sbs = core.cri_list(k.cri_socket)
        assert [c["id"] for c in cs] == ["cid123"] and [s["name"] for s in sbs] == ["p"]
        cs, _ = core.cri_list(k.cri_socket)  # remembered: straight to v1alpha2
        assert len(cs) == 1
