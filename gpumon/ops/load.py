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
* ``partial`` — a quarter of the CUs burning (partial-occupancy validation);
* ``pcie``  — DMA copies between pinned host memory and the device (``pcie_direction`` ``h2d`` /
  ``d2h`` / ``both`` on two streams): the host link's known traffic, against which
  ``gpu_pcie_bandwidth_bytes_per_second`` is checked (native ``PcieLoad``; ``stats()`` gives
  ``h2d_bytes`` / ``d2h_bytes`` and ``GBps_wall``, no FLOPs).

``period_s`` > 0 turns ``duty`` into long bursts (``duty * period_s`` busy, then idle to the end
of the period: a training step's compute / communication phases) instead of an idle gap after
every batch.

``mfma_dtype`` swaps the bf16 burn for another matrix path of the same geometry
(``csrc/hip/burn_dtypes.hip``): ``f16``, ``fp8``, ``f32``, ``f64``, ``i8`` and the block-scaled
``mxfp8`` / ``mxfp4`` (f8f6f4) instructions — one load per ``gpu_mfma_tflops{dtype}`` counter.
"""

from __future__ import annotations

from .._native import hip

KINDS = ("mfma", "hbm", "mixed", "concurrent", "partial", "pcie")
PCIE_DIRECTIONS = ("h2d", "d2h", "both")
DTYPES = ("bf16", "f16", "fp8", "f32", "f64", "i8", "mxfp8", "mxfp4")


class SyntheticLoad:
    def __init__(self, dev: int = 0, kind: str = "mixed", duty: float = 1.0, hbm_bytes: int = 1 << 30,
                 mfma_iters: int = 8192, mfma_shape: int = 16, mfma_dtype: str = "bf16", period_s: float = 0.0,
                 pcie_direction: str = "both", pcie_bytes: int = 256 << 20):
        if kind not in KINDS:
            raise ValueError(f"load kind {kind!r}: one of {', '.join(KINDS)}")
        if mfma_dtype not in DTYPES:
            raise ValueError(f"mfma_dtype {mfma_dtype!r}: one of {', '.join(DTYPES)}")
        if not 0.0 < duty <= 1.0:
            raise ValueError(f"duty {duty}: in (0, 1]")
        if mfma_shape not in (16, 32):
            raise ValueError(f"mfma_shape {mfma_shape}: 16 or 32")
        if kind == "pcie":
            if pcie_direction not in PCIE_DIRECTIONS:
                raise ValueError(f"pcie_direction {pcie_direction!r}: one of {', '.join(PCIE_DIRECTIONS)}")
            self._g = hip().PcieLoad(dev, pcie_bytes, pcie_direction, duty)
        else:
            self._g = hip().LoadGen(dev, kind, duty, hbm_bytes, mfma_iters, mfma_shape, mfma_dtype, period_s)
        self.dev = dev
        self.kind = kind

    @staticmethod
    def rates(a: dict, b: dict) -> dict:
        """The load's event-timed rates between two ``stats()`` snapshots: TFLOP/s over the MFMA
        batches' GPU time, TB/s over the HBM batches' GPU time (each counts only while its own kernel
        kind ran, so a mixed load's phases are not averaged in), and ``busy`` = GPU time / wall time
        (the duty the GPU saw). ``tflops_wall`` / ``tbps_wall``: the same work over wall time, which
        adds up across processes sharing one GPU (the kernel-time rates do not: one process's MFMA
        kernels run while another's HBM kernels do)."""
        wall = b["wall_s"] - a["wall_s"]
        if "h2d_bytes" in b:  # pcie: link bytes over wall time, per direction
            return {"tflops": 0.0, "tbps": 0.0, "busy": (b["busy_s"] - a["busy_s"]) / wall if wall > 0 else 0.0,
                    "h2d_GBps": (b["h2d_bytes"] - a["h2d_bytes"]) / wall / 1e9 if wall > 0 else 0.0,
                    "d2h_GBps": (b["d2h_bytes"] - a["d2h_bytes"]) / wall / 1e9 if wall > 0 else 0.0}
        dm, dh = b["mfma_s"] - a["mfma_s"], b["hbm_s"] - a["hbm_s"]
        return {"tflops": (b["flops"] - a["flops"]) / dm / 1e12 if dm > 0 else 0.0,
                "tbps": (b["bytes"] - a["bytes"]) / dh / 1e12 if dh > 0 else 0.0,
                "busy": (b["busy_s"] - a["busy_s"]) / wall if wall > 0 else 0.0,
                "tflops_wall": (b["flops"] - a["flops"]) / wall / 1e12 if wall > 0 else 0.0,
                "tbps_wall": (b["bytes"] - a["bytes"]) / wall / 1e12 if wall > 0 else 0.0}

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
