"""HIP ordinal -> exporter device by PCI BDF (gpumon/parallel/devmap.py).

A process under HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES numbers its GPUs 0..n-1 while the
exporter's gpu_id is the node-wide hip_id, so the bench, the xGMI validator and the multi-GPU tests
pair the two by BDF. Here the real AmdSmiBackend and RocmSmiBackend run over the fake vendor
libraries with 8 GPUs; the HIP side is what hipDeviceGetPCIBusId reports under each visibility
setting (ordinal k = the k-th listed node GPU), written out as ordinal -> BDF dicts. The reference
numbered GPUs by CLI output order (/root/reference/gpu.py:119-120)."""

import os

import pytest

from conftest import make_locked
from gpumon.export import promtext
from gpumon.parallel.devmap import DeviceMapError, index_of, match, normalize_bdf, positional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE_AMDSMI = os.path.join(ROOT, "build", "fakes", "libfake_amd_smi.so")
FAKE_RSMI = os.path.join(ROOT, "build", "fakes", "libfake_rocm_smi.so")


@pytest.fixture(scope="module", autouse=True)
def fakes():
    make_locked("fakes")


@pytest.fixture
def exporter(core, monkeypatch):
    made = []

    def make(backend, devices=(), gpus=8):
        monkeypatch.setenv("FAKE_AMDSMI_GPUS", str(gpus))
        monkeypatch.setenv("FAKE_RSMI_GPUS", str(gpus))
        cfg = {"backend": backend, "serve_http": False, "interval_s": 0, "verify_kfd": False, "init_retry_s": 0.0,
               "devices": list(devices), "fast_path": False}
        cfg["amdsmi_lib" if backend == "amdsmi" else "rocm_smi_lib"] = FAKE_AMDSMI if backend == "amdsmi" else FAKE_RSMI
        ex = core.Exporter(cfg)
        assert ex.start() == ""
        made.append(ex)
        return ex

    yield make
    for ex in made:
        ex.stop()


def test_normalize_bdf():
    assert normalize_bdf("0000:75:00.0") == "0000:75:00.0"
    assert normalize_bdf("75:00.0") == "0000:75:00.0"
    assert normalize_bdf(" 0001:E5:1f.7 ") == "0001:e5:1f.7"
    for bad in ("", "3", "75:00", "0000:75:20.0", "0000:75:00.8", "zz:00.0", "0000:75:00.0x"):
        assert normalize_bdf(bad) == "", bad


def _node_bdfs(exporter, backend):
    st = exporter(backend).statics()
    assert [s["hip_id"] for s in st] == list(range(8))
    return [s["bdf"] for s in st]


@pytest.mark.parametrize("backend", ["amdsmi", "rocm_smi"])
@pytest.mark.parametrize("visible", [[3, 5], [6, 2], [7], list(range(8))],
                         ids=["hip_visible_3_5", "rocr_visible_6_2", "one_of_8", "all"])
def test_visible_subset_maps_to_node_gpus(exporter, backend, visible):
    """HIP_VISIBLE_DEVICES=3,5: ordinals 0,1 are node GPUs 3,5. ROCR_VISIBLE_DEVICES=6,2: ordinal 0
    is node GPU 6 (the listed order), so ordinal order and the exporter's hip_id order differ."""
    node = _node_bdfs(exporter, backend)
    hip = {k: node[g].upper() for k, g in enumerate(visible)}  # what each ordinal's hipDeviceGetPCIBusId says
    ex = exporter(backend, devices=[hip[k] for k in sorted(hip)])
    rows = match(hip, ex.statics())
    assert [r["gpu_id"] for r in rows] == [str(g) for g in visible]
    for r in rows:  # the index points at the sampled device with that identity
        assert ex.statics()[r["index"]]["bdf"] == normalize_bdf(hip[r["hip_ordinal"]])
        assert ex.statics()[r["index"]]["gpu_id"] == r["gpu_id"]
    ex.tick()
    fam = promtext.parse(ex.metrics_text())  # what the scrape says: exactly the loaded GPUs
    assert sorted(l["gpu_id"] for _, l, _ in fam["node_gpu_gpu_util"]["samples"]) == sorted(str(g) for g in visible)
    assert sorted(index_of(rows).values()) == list(range(len(visible)))


@pytest.mark.parametrize("backend", ["amdsmi", "rocm_smi"])
def test_range_n_was_wrong_for_a_non_prefix_subset(exporter, backend):
    """What round 3 did (devices=range(n)) samples node GPUs 0,1 for a job on GPUs 3,5: the BDF
    match refuses that exporter instead of silently pairing the wrong GPUs."""
    node = _node_bdfs(exporter, backend)
    hip = {0: node[3], 1: node[5]}
    wrong = exporter(backend, devices=[0, 1])
    assert [s["gpu_id"] for s in wrong.statics()] == ["0", "1"]
    with pytest.raises(DeviceMapError, match="HIP ordinal 0"):
        match(hip, wrong.statics())


def test_rocm_smi_fallback_index_order_is_the_hip_id(exporter):
    """The rocm_smi fallback exports its enumeration index as hip_id; filtered by BDF it keeps the
    node-wide index, the same gpu_id libamd_smi gives the GPU."""
    a = {s["bdf"]: s["gpu_id"] for s in exporter("amdsmi").statics()}
    r = {s["bdf"]: s["gpu_id"] for s in exporter("rocm_smi").statics()}
    assert a == r
    bdf4 = [b for b, g in r.items() if g == "4"][0]
    ex = exporter("rocm_smi", devices=[bdf4])
    assert [s["gpu_id"] for s in ex.statics()] == ["4"]


def test_replicas_and_positional(core):
    st = [{"index": i, "gpu_id": str(i), "bdf": "0000:05:00.0"} for i in range(3)]  # replicate=3 of one GPU
    with pytest.raises(DeviceMapError):
        match({0: "05:00.0"}, st)
    assert match({0: "05:00.0"}, st, replicas=True)[0]["index"] == 0
    assert [r["gpu_id"] for r in positional(2, st)] == ["0", "1"]
    with pytest.raises(DeviceMapError):
        positional(4, st)


def test_native_config_accepts_bdfs(tmp_path):
    """bin/gpumon-exporter --devices takes hip ids and BDFs; a token that is neither is an error."""
    import subprocess

    make_locked("core")
    exe = os.path.join(ROOT, "bin", "gpumon-exporter")
    r = subprocess.run([exe, "--devices", "2,75:00.0", "--print-config"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    import json

    assert json.loads(r.stdout)["devices"] == ["2", "0000:75:00.0"]
    r = subprocess.run([exe, "--devices", "gpu3", "--print-config"], capture_output=True, text=True, timeout=30)
    assert r.returncode != 0 and "neither a hip id nor a PCI BDF" in r.stderr
