"""xGMI traffic generators used to validate the per-link xGMI counters.

* :func:`allreduce_step` — one RCCL ring all-reduce over the job's process group (backend "nccl"
  is RCCL on ROCm). On an 8x MI355X node a ring touches every GPU's links; ring collectives are
  per-link bound (7 links x ~153 GB/s bidirectional per GPU), so the per-link rate the exporter
  reports should approach 2*(N-1)/N * bytes / t spread over the ring's links.
* :class:`PeerCopier` — hipMemcpyPeerAsync-equivalent (torch ``copy_`` between devices) from one
  GPU to one peer: drives exactly one link, to check the link index -> peer BDF mapping.
Neither is used by the exporter itself; they are validation load only.
"""

from __future__ import annotations

import time
from typing import Optional


def allreduce_step(buf, group=None) -> float:
    """All-reduce ``buf`` in place; returns seconds (includes a device sync)."""
    import torch
    import torch.distributed as dist

    t0 = time.perf_counter()
    dist.all_reduce(buf, group=group)
    if buf.is_cuda:
        torch.cuda.synchronize(buf.device)
    return time.perf_counter() - t0


def allreduce_busbw(nbytes: int, seconds: float, world: int) -> float:
    """Ring all-reduce bus bandwidth (bytes/s): 2*(N-1)/N * size / t (nccl-tests convention)."""
    if seconds <= 0 or world <= 1:
        return 0.0
    return 2.0 * (world - 1) / world * nbytes / seconds


class PeerCopier:
    def __init__(self, src_dev: int, dst_dev: int, nbytes: int = 1 << 30):
        import torch

        self.src = torch.empty(nbytes // 4, dtype=torch.float32, device=f"cuda:{src_dev}")
        self.dst = torch.empty(nbytes // 4, dtype=torch.float32, device=f"cuda:{dst_dev}")
        self.nbytes = nbytes

    def run(self, seconds: float = 1.0) -> float:
        """Copy repeatedly for ~``seconds``; returns achieved bytes/s."""
        import torch

        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < seconds:
            self.dst.copy_(self.src, non_blocking=True)
            n += 1
            if n % 8 == 0:
                torch.cuda.synchronize(self.src.device)
        torch.cuda.synchronize(self.src.device)
        return n * self.nbytes / (time.perf_counter() - t0)


def make_allreduce_buffer(nbytes: int, device) -> Optional[object]:
    import torch

    return torch.ones(max(1, nbytes // 2), dtype=torch.bfloat16, device=device)
