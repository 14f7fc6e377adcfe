#!/usr/bin/env python3
"""Interleaved A/B microbenchmark of the K2 kernels on one MI355X (rule: variants timed in rounds in
ONE process, report median/min). Prints JSON. Used to choose the HBM-stream unroll / grid."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gpumon import hip  # noqa: E402

H = hip()
cus = H.device_cu_count(0)
s = torch.cuda.current_stream().cuda_stream
nbytes = 2 << 30
x = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda").fill_(1.0)
y = torch.empty_like(x)
n16 = nbytes // 16
variants = [(u, b) for u in (1, 2, 4, 8) for b in (cus * 4, cus * 8, cus * 16, cus * 32)]
res = {f"u{u}_b{b}": [] for u, b in variants}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3):  # warm
    for u, b in variants:
        H.stream_copy(0, x.data_ptr(), y.data_ptr(), n16, b, s, u)
torch.cuda.synchronize()
for rnd in range(7):
    for u, b in variants:
        e0.record()
        for _ in range(4):
            H.stream_copy(0, x.data_ptr(), y.data_ptr(), n16, b, s, u)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 4
        res[f"u{u}_b{b}"].append(2 * nbytes / (ms * 1e-3) / 1e12)
out = {"stream_copy_TBps": {k: {"median": statistics.median(v), "max": max(v)} for k, v in res.items()}}
# MFMA burn at a few occupancies
a = (torch.randn(32, 16) * 0.1).to(torch.bfloat16).cuda()
bm = (torch.randn(16, 32) * 0.1).to(torch.bfloat16).cuda()
o = torch.zeros(cus * 32 * 4, device="cuda")
burn = {}
for blocks in (cus, cus * 2, cus * 4, cus * 8):
    t = []
    for rnd in range(5):
        e0.record()
        H.mfma_burn(0, a.data_ptr(), bm.data_ptr(), o.data_ptr(), blocks, 4096, s)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        t.append(blocks * 4 * 4 * 4096 * 32768 / (ms * 1e-3) / 1e12)
    burn[f"blocks_{blocks}"] = {"median": statistics.median(t), "max": max(t)}
out["mfma_burn_TFLOPs"] = burn
print(json.dumps(out))
