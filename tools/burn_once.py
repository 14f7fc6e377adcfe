#!/usr/bin/env python3
"""Run K2 kernels a fixed number of times (for rocprofv3 --pmc cross-checks of the PMC module)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gpumon import hip  # noqa: E402

H = hip()
a = (torch.randn(32, 16) * 0.1).to(torch.bfloat16).cuda()
b = (torch.randn(16, 32) * 0.1).to(torch.bfloat16).cuda()
out = torch.zeros(2048 * 4, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    H.mfma_burn(0, a.data_ptr(), b.data_ptr(), out.data_ptr(), 2048, 8192, s)
x = torch.empty(1 << 28, device="cuda")
y = torch.empty_like(x)
for _ in range(20):
    H.stream_copy(0, x.data_ptr(), y.data_ptr(), x.numel() // 4, 4096, s)
torch.cuda.synchronize()
print("ok")
