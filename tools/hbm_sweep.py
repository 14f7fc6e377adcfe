#!/usr/bin/env python3
"""HBM stream-copy sweep on one MI355X: cache policy (nt / plain loads and stores) x unroll x grid x
grid-stride vs contiguous spans. Interleaved rounds in ONE process, 2 GiB + 2 GiB buffers (8x the
256 MiB Infinity Cache), bytes = read + write. Prints JSON sorted by median TB/s."""
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
if len(sys.argv) > 1 and sys.argv[1] == "--short":  # finalists + vendor baselines
    # one chunk per workgroup (span == chunk: the grid covers the buffer once, no loop), as PyTorch's
    # elementwise kernels launch, vs the grid-stride finalists
    variants = [(u, n16 // (256 * u), pol, True) for u in (1, 2, 4) for pol in (0, 1, 2, 3)]
    variants += [(4, cus * 64, 0, False), "torch_copy", "torch_mul_out"]
else:
    variants = [(u, b, pol, span) for u in (2, 4, 8) for b in (cus * 8, cus * 32) for pol in (0, 1, 2, 3)
                for span in (False, True)]
    variants += [(4, cus * 64, 0, False), (4, cus * 64, 1, False), (4, cus * 16, 0, False), (4, cus * 16, 1, False)]
name = lambda v: v if isinstance(v, str) else f"u{v[0]}_b{v[1]}_p{v[2]}_{'span' if v[3] else 'grid'}"  # noqa: E731


def run(v):
    if v == "torch_copy":
        y.copy_(x)
    elif v == "torch_mul_out":  # PyTorch's own elementwise kernel, same bytes
        torch.mul(x, 1.0, out=y)
    else:
        H.stream_copy(0, x.data_ptr(), y.data_ptr(), n16, v[1], s, v[0], v[2], v[3])
res = {name(v): [] for v in variants}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for v in variants:  # warm + compile
    run(v)
torch.cuda.synchronize()
assert torch.equal(x[:1024], y[:1024]) and torch.equal(x[-1024:], y[-1024:])
for rnd in range(9 if len(variants) < 10 else 5):
    for v in variants:
        e0.record()
        for _ in range(3):
            run(v)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 3
        res[name(v)].append(2 * nbytes / (ms * 1e-3) / 1e12)
    print(f"round {rnd} done", file=sys.stderr, flush=True)
out = sorted(({"variant": k, "median": round(statistics.median(t), 3), "max": round(max(t), 3)} for k, t in res.items()),
             key=lambda r: -r["median"])
print(json.dumps({"cus": cus, "bytes_per_launch": 2 * nbytes, "results": out}))
