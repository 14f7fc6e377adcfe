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


# ------------------------------------------------------------------------------------------------
# Link-map validation: drive one peer copy at a time and see which link counter moves.
# ------------------------------------------------------------------------------------------------
def busiest_link(rates: dict, key: str = "xgmi_wr_Bps"):
    """(link index, bytes/s) of the link carrying the most traffic in one device's rate dict."""
    vals = rates.get(key) or []
    if not vals:
        return -1, 0.0
    k = max(range(len(vals)), key=lambda i: vals[i])
    return k, float(vals[k])


def link_peer_bdf(sample: dict, link: int) -> str:
    links = sample.get("links") or []
    return links[link].get("peer_bdf", "") if 0 <= link < len(links) else ""


def validate_pair(ex, src: int, dst: int, copier_factory=None, seconds: float = 2.0,
                  interval: float = 0.1) -> dict:
    """Copy src -> dst for ``seconds`` while the exporter ``ex`` samples both devices; report the
    copy bandwidth, the link on ``src`` whose write counter moved most, the peer BDF the exporter
    attributes to that link and whether it is ``dst``'s BDF."""
    statics = {s["index"]: s for s in ex.statics()}
    copier = (copier_factory or PeerCopier)(src, dst)
    seq0 = ex.seq
    ex.wait_for_seq(seq0 + 1, 10.0)
    result = {"src": src, "dst": dst}
    stop = time.perf_counter() + seconds
    best = (-1, 0.0)
    rx = (-1, 0.0)
    bw = []
    while time.perf_counter() < stop:
        bw.append(copier.run(min(interval * 3, max(0.05, stop - time.perf_counter()))))
        r = ex.rates()
        if src < len(r) and r[src].get("valid"):
            cand = busiest_link(r[src], "xgmi_wr_Bps")
            if cand[1] > best[1]:
                best = cand
        if dst < len(r) and r[dst].get("valid"):
            cand = busiest_link(r[dst], "xgmi_rd_Bps")
            if cand[1] > rx[1]:
                rx = cand
    samples = ex.samples()
    result["copy_GBps"] = round(sum(bw) / max(1, len(bw)) / 1e9, 2)
    result["src_link"], result["src_link_tx_GBps"] = best[0], round(best[1] / 1e9, 2)
    result["dst_link"], result["dst_link_rx_GBps"] = rx[0], round(rx[1] / 1e9, 2)
    peer = link_peer_bdf(samples[src], best[0]) if src < len(samples) else ""
    result["src_link_peer_bdf"] = peer
    result["dst_bdf"] = statics.get(dst, {}).get("bdf", "")
    result["peer_matches"] = bool(peer) and peer.lower() == result["dst_bdf"].lower()
    return result
