"""K2 load API (gpumon/ops/load.py) on CPU: argument checks happen before any HIP call, and the
event-timed rates between two stats snapshots count each kernel kind over its own GPU time."""

import pytest

from gpumon.ops.load import SyntheticLoad


@pytest.mark.parametrize("kw,msg", [({"kind": "burn"}, "load kind"), ({"mfma_dtype": "bf8"}, "mfma_dtype"),
                                    ({"duty": 0.0}, "duty"), ({"duty": 1.5}, "duty"), ({"mfma_shape": 8}, "mfma_shape")])
def test_bad_arguments_are_refused_before_the_gpu(kw, msg):
    with pytest.raises(ValueError, match=msg):
        SyntheticLoad(**kw)


def test_rates_use_each_kinds_own_gpu_time():
    a = {"flops": 0.0, "bytes": 0.0, "mfma_s": 1.0, "hbm_s": 1.0, "busy_s": 2.0, "wall_s": 2.0}
    # a mixed load over 2 s of wall time: 0.9 s of MFMA batches at 2 PFLOP/s, 0.9 s of HBM at 6 TB/s
    b = {"flops": 1.8e15, "bytes": 5.4e12, "mfma_s": 1.9, "hbm_s": 1.9, "busy_s": 3.8, "wall_s": 4.0}
    r = SyntheticLoad.rates(a, b)
    assert r["tflops"] == pytest.approx(2000.0) and r["tbps"] == pytest.approx(6.0) and r["busy"] == pytest.approx(0.9)
    # over wall time (what adds up across processes sharing a GPU): 1.8e15 / 2 s, 5.4e12 / 2 s
    assert r["tflops_wall"] == pytest.approx(900.0) and r["tbps_wall"] == pytest.approx(2.7)
    assert SyntheticLoad.rates(a, a) == {"tflops": 0.0, "tbps": 0.0, "busy": 0.0, "tflops_wall": 0.0, "tbps_wall": 0.0}
