"""K2 synthetic HIP load used to validate the exporter under known conditions (bench + GPU tests).

``SyntheticLoad(dev, kind)`` drives one GPU from a native C++ thread (no GIL) with back-to-back
launches of the gfx950 kernels in ``csrc/hip/kernels.hip``:

* ``mfma``  — bf16 MFMA burn: ``mfma_shape=16`` = ``v_mfma_f32_16x16x32_bf16`` x 8 chains per wave
  (2.24 PFLOP/s sustained on MI355X, profiles/r1_kernels_and_pmc.md), ``32`` =
  ``v_mfma_f32_32x32x16_bf16`` x 4 chains (1.76–2.0 PFLOP/s: the chip holds a lower clock on it);
* ``hbm``   — 16 B/lane non-temporal copy over a ``hbm_bytes`` buffer pair, one 4 KiB chunk per
  workgroup (6.5 TB/s on MI355X, profiles/r1_hbm_stream.md);
* ``mixed`` — MFMA and HBM batches ALTERNATING on one stream (time-sliced: each rate holds only
  during its own phase, never both at once); ``duty`` < 1 inserts idle gaps;
* ``concurrent`` — the MFMA burn and the HBM stream on two streams at the same time (both pipes
  loaded at once: the power / thermal worst case); ``stats()["tflops_wall"]`` /
  ``["tbps_wall"]`` are the rates averaged over wall time;
* ``partial`` — a quarter of the CUs burning (partial-occupancy validation).

``period_s`` > 0 turns ``duty`` into long bursts (``duty * period_s`` busy, then idle to the end
of the period: a training step's compute / communication phases) instead of an idle gap after
every batch.

``mfma_dtype`` swaps the bf16 burn for another matrix path of the same geometry
(``csrc/hip/burn_dtypes.hip``): ``f16``, ``fp8``, ``f32``, ``f64``, ``i8`` and the block-scaled
``mxfp8`` / ``mxfp4`` (f8f6f4) instructions — one load per ``gpu_mfma_tflops{dtype}`` counter.
"""

from __future__ import annotations

from .._native import hip


class SyntheticLoad:
    def __init__(self, dev: int = 0, kind: str = "mixed", duty: float = 1.0, hbm_bytes: int = 1 << 30,
                 mfma_iters: int = 8192, mfma_shape: int = 16, mfma_dtype: str = "bf16", period_s: float = 0.0):
        self._g = hip().LoadGen(dev, kind, duty, hbm_bytes, mfma_iters, mfma_shape, mfma_dtype, period_s)
        self.dev = dev
        self.kind = kind

    def start(self) -> "SyntheticLoad":
        self._g.start()
        return self

    def stop(self) -> None:
        self._g.stop()

    def stats(self) -> dict:
        return self._g.stats()

    def __enter__(self):
        return self.start()

    def __exit__(self, *a):
        self.stop()
