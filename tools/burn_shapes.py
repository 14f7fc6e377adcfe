#!/usr/bin/env python3
"""Sustained bf16 MFMA burn throughput per MFMA shape (LoadGen, back-to-back launches, steady DVFS
clock): v_mfma_f32_32x32x16_bf16 x4 chains vs v_mfma_f32_16x16x32_bf16 x8 chains. Prints JSON."""

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from gpumon import hip

    H = hip()
    out = {}
    for shape in (32, 16, 32, 16):
        g = H.LoadGen(0, "mfma", 1.0, 1 << 20, 8192, shape)
        g.start()
        time.sleep(1.5)          # reach the steady clock
        s0 = g.stats()
        time.sleep(3.0)
        s1 = g.stats()
        g.stop()
        tf = (s1["flops"] - s0["flops"]) / max(1e-9, s1["mfma_s"] - s0["mfma_s"]) / 1e12
        out.setdefault(f"shape_{shape}", []).append(round(tf, 1))
        time.sleep(1.0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
