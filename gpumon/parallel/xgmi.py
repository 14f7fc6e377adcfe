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
from typing import Dict, Optional


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
    """One GPU pushing into one peer's memory, back to back, from a native thread (``_hip.XgmiLoad``:
    a copy kernel on ``src`` whose stores cross the src->dst xGMI link, or ``method="dma"`` for
    hipMemcpyPeerAsync). ``run(seconds)`` keeps it running and returns the bytes/s achieved over
    that window; ``close()`` stops it."""

    def __init__(self, src_dev: int, dst_dev: int, nbytes: int = 256 << 20, method: str = "kernel",
                 blocks: int = 512):
        from .._native import hip

        self._g = hip().XgmiLoad(src_dev, dst_dev, nbytes, method, blocks)
        self.src, self.dst, self.nbytes = src_dev, dst_dev, nbytes
        self._started = False

    def start(self) -> "PeerCopier":
        if not self._started:
            self._g.start()
            self._started = True
        return self

    def stats(self) -> dict:
        return self._g.stats()

    def run(self, seconds: float = 1.0) -> float:
        self.start()
        s0 = self._g.stats()
        time.sleep(seconds)
        s1 = self._g.stats()
        dt = s1["wall_s"] - s0["wall_s"]
        return (s1["bytes"] - s0["bytes"]) / dt if dt > 0 else 0.0

    def close(self) -> None:
        if self._started:
            self._g.stop()
            self._started = False


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


def _median(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2] if xs else 0.0


def validate_pair(ex, src: int, dst: int, copier_factory=None, seconds: float = 2.0,
                  interval: float = 0.1, index_of: Optional[Dict[int, int]] = None) -> dict:
    """Copy src -> dst for ``seconds`` while the exporter ``ex`` samples both devices. Reports the
    copy bandwidth, the link on ``src`` whose write counter moved most (the mode over the sampled
    ticks), the median exporter rate on that link (``src_link_tx_GBps``) and its ratio to the copy
    rate (``tx_vs_copy``), the same on the receiving side, the peer BDF the exporter attributes to
    the src link and whether it is ``dst``'s BDF (``peer_matches``). The first tick after the
    copy starts is skipped: its rate spans time before the copy.

    ``src`` / ``dst`` are HIP ordinals (what the copier loads). ``index_of`` maps them to the
    exporter's device indices; by default they are paired by PCI BDF (gpumon/parallel/devmap.py)
    when the real copier runs, and taken as equal for an injected ``copier_factory`` (mock)."""
    if index_of is None:
        if copier_factory is None:
            from .devmap import exporter_rows
            from .devmap import index_of as _index_of

            index_of = _index_of(exporter_rows(ex, sorted({src, dst})))
        else:
            index_of = {src: src, dst: dst}
    si, di = index_of[src], index_of[dst]
    statics = {s["index"]: s for s in ex.statics()}
    copier = (copier_factory or PeerCopier)(src, dst)
    result = {"src": src, "dst": dst, "src_gpu_id": statics.get(si, {}).get("gpu_id"),
              "dst_gpu_id": statics.get(di, {}).get("gpu_id")}
    bw, tx, rx = [], [], []  # per poll: copy B/s; (link, B/s) busiest on src write / dst read
    try:
        bw_first = copier.run(min(interval * 2, 1.0))  # ramp: the tick spanning the start is discarded
        seq = ex.seq
        ex.wait_for_seq(seq + 1, interval * 5 + 5.0)
        stop = time.perf_counter() + seconds
        while time.perf_counter() < stop:
            bw.append(copier.run(min(interval * 2, max(0.05, stop - time.perf_counter()))))
            r = ex.rates()
            if si < len(r) and r[si].get("valid"):
                tx.append(busiest_link(r[si], "xgmi_wr_Bps"))
            if di < len(r) and r[di].get("valid"):
                rx.append(busiest_link(r[di], "xgmi_rd_Bps"))
    finally:
        close = getattr(copier, "close", None)
        if close:
            close()
    samples = ex.samples()

    def mode_link(xs):
        links = [k for k, v in xs if k >= 0 and v > 0]
        if not links:
            return -1, 0.0
        k = max(set(links), key=links.count)
        return k, _median([v for kk, v in xs if kk == k])

    copy_bps = sum(bw) / len(bw) if bw else bw_first
    result["copy_GBps"] = round(copy_bps / 1e9, 2)
    (sl, sv), (dl, dv) = mode_link(tx), mode_link(rx)
    result["src_link"], result["src_link_tx_GBps"] = sl, round(sv / 1e9, 2)
    result["dst_link"], result["dst_link_rx_GBps"] = dl, round(dv / 1e9, 2)
    result["tx_vs_copy"] = round(sv / copy_bps, 3) if copy_bps > 0 else None
    result["rx_vs_copy"] = round(dv / copy_bps, 3) if copy_bps > 0 else None
    peer = link_peer_bdf(samples[si], sl) if si < len(samples) else ""
    result["src_link_peer_bdf"] = peer
    result["dst_bdf"] = statics.get(di, {}).get("bdf", "")
    result["peer_matches"] = bool(peer) and peer.lower() == result["dst_bdf"].lower()
    return result


def rate_within(r: dict, tol: float = 0.15) -> bool:
    """The exporter's per-link tx rate agrees with the copy's own rate within ``tol``."""
    v = r.get("tx_vs_copy")
    return v is not None and abs(v - 1.0) <= tol
