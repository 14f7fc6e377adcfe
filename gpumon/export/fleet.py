"""Fleet view over running exporters: ``gpumon top --url URL [--url URL ...]``.

The reference's only views were Grafana boards over InfluxDB (``img/grafana.png``: per-node,
per-card VRAM and utilisation gauges; the 2019 screenshot's container table). This renders the same
two tables in a terminal from any number of node exporters' ``/metrics``, without opening a GPU (the
DaemonSet already samples it): one HTTP GET per node through the native client, parsed with the
strict text-format parser.
"""

from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Optional, Tuple

from . import promtext

Key = Tuple[str, str]  # (host, gpu_id)


def _per_gpu(fam: dict, name: str, **match) -> Dict[Key, float]:
    out: Dict[Key, float] = {}
    for n, labels, v in fam.get(name, {"samples": []})["samples"]:
        if n != name or any(labels.get(k) != str(x) for k, x in match.items()):
            continue
        out[(labels.get("host", "?"), labels.get("gpu_id", "?"))] = v
    return out


def gpu_rows(fam: dict) -> List[dict]:
    """One dict per (host, gpu_id) seen in a parsed exposition."""
    util = _per_gpu(fam, "node_gpu_gpu_util")
    used = _per_gpu(fam, "gpu_vram_used_bytes")
    total = _per_gpu(fam, "gpu_vram_total_bytes")
    power = _per_gpu(fam, "gpu_power_watts")
    hot = _per_gpu(fam, "gpu_temperature_celsius", sensor="hotspot")
    gfx = _per_gpu(fam, "gpu_clock_mhz", clock="gfx")
    up = _per_gpu(fam, "gpu_up")
    mfma = _per_gpu(fam, "gpu_mfma_util_percent")
    active = _per_gpu(fam, "gpu_active_processes")
    pcie = _per_gpu(fam, "gpu_pcie_bandwidth_bytes_per_second")
    xcd: Dict[Key, Dict[int, float]] = defaultdict(dict)
    for n, labels, v in fam.get("gpu_xcd_busy_percent", {"samples": []})["samples"]:
        xcd[(labels.get("host", "?"), labels.get("gpu_id", "?"))][int(labels.get("xcd", 0))] = v
    ue: Dict[Key, float] = defaultdict(float)
    for n, labels, v in fam.get("gpu_ecc_errors_total", {"samples": []})["samples"]:
        if labels.get("type") == "uncorrectable":
            ue[(labels.get("host", "?"), labels.get("gpu_id", "?"))] += v
    keys = sorted(set(util) | set(up) | set(used), key=lambda k: (k[0], int(k[1]) if k[1].isdigit() else 1 << 30, k[1]))
    rows = []
    for k in keys:
        rows.append({"host": k[0], "gpu_id": k[1], "up": up.get(k), "util": util.get(k),
                     "xcd": [xcd[k][i] for i in sorted(xcd[k])] if k in xcd else [],
                     "vram_used": used.get(k), "vram_total": total.get(k), "power": power.get(k),
                     "hot": hot.get(k), "gfx_mhz": gfx.get(k), "ecc_ue": ue.get(k) if k in ue else None,
                     "mfma": mfma.get(k), "procs": active.get(k), "pcie_Bps": pcie.get(k)})
    return rows


def pod_rows(fam: dict) -> List[dict]:
    """pod_gpu series (active processes and idle allocations) joined on their labels."""
    mem = fam.get("pod_gpu_used_memory_bytes", {"samples": []})["samples"]
    occ = {tuple(sorted(l.items())): v for _, l, v in fam.get("pod_gpu_proc_cu_occupancy_percent",
                                                               {"samples": []})["samples"]}
    queues = {tuple(sorted(l.items())): v for _, l, v in fam.get("pod_gpu_proc_queues", {"samples": []})["samples"]}
    rows = []
    for _, labels, v in mem:
        k = tuple(sorted(labels.items()))
        rows.append(dict(labels, used_memory_bytes=v, cu_pct=occ.get(k), queues=queues.get(k)))
    rows.sort(key=lambda r: (r.get("host", ""), r.get("gpu_id", ""), r.get("namespace", ""), r.get("podname", "")))
    return rows


def _f(v: Optional[float], w: int, p: int = 0) -> str:
    return "-".rjust(w) if v is None else f"{v:{w}.{p}f}"


def sharing_label(n: Optional[float]) -> str:
    """The sharing state from `gpu_active_processes` (idle / one process / shared by N): the
    reference's gauge board marked its node columns "(共享)" shared / "(独占)" exclusive
    (/root/reference/img/grafana.png)."""
    if n is None:
        return "-"
    return "idle" if n < 1 else ("exclusive" if n < 2 else f"shared:{int(n)}")


def render(frames: List[dict], errors: Optional[Dict[str, str]] = None) -> str:
    """Text tables for parsed expositions (one per node)."""
    lines = [f"{'HOST':<20}{'GPU':>4} {'UP':>2} {'UTIL%':>6} {'XCD busy% (0-7)':<32} {'VRAM GiB':>13} "
             f"{'PWR W':>6} {'HOT C':>6} {'GFX MHz':>8} {'MFMA%':>6} {'PCIe GB/s':>9} {'ECC-UE':>7} {'SHARING':>10}"]
    pods = []
    for fam in frames:
        for r in gpu_rows(fam):
            xcd = " ".join(f"{int(x):3d}" for x in r["xcd"][:8]) if r["xcd"] else "-"
            vram = "-" if r["vram_used"] is None else f"{r['vram_used'] / 2**30:.1f}/{(r['vram_total'] or 0) / 2**30:.0f}"
            lines.append(f"{r['host'][:19]:<20}{r['gpu_id']:>4} {_f(r['up'], 2)} {_f(r['util'], 6)} {xcd:<32} "
                         f"{vram:>13} {_f(r['power'], 6)} {_f(r['hot'], 6)} {_f(r['gfx_mhz'], 8)} "
                         f"{_f(r['mfma'], 6, 1)} "
                         f"{_f(None if r['pcie_Bps'] is None else r['pcie_Bps'] / 1e9, 9, 2)} "
                         f"{_f(r['ecc_ue'], 7)} {sharing_label(r['procs']):>10}")
        pods.extend(pod_rows(fam))
    for url, err in (errors or {}).items():
        lines.append(f"{url}: {err}")
    lines.append("")
    lines.append(f"{'HOST':<20}{'GPU':>4} {'NAMESPACE':<14}{'POD':<32}{'USER':<10}{'PID':>8} {'MEM MiB':>9} "
                 f"{'CU%':>6} {'Q':>3}  PROCESS")
    for p in pods:
        lines.append(f"{p.get('host', '?')[:19]:<20}{p.get('gpu_id', '?'):>4} {p.get('namespace', '-')[:13]:<14}"
                     f"{p.get('podname', '-')[:31]:<32}{p.get('user_name', '-')[:9]:<10}{p.get('pid', '-'):>8} "
                     f"{p['used_memory_bytes'] / 1048576:9.0f} {_f(p['cu_pct'], 6, 1)} {_f(p.get('queues'), 3)}  "
                     f"{p.get('procressname', '-')[:30]}")
    return "\n".join(lines)


def fetch(urls: List[str], timeout_s: float = 3.0, workers: int = 16,
          ca_file: str = "", token: str = "") -> Tuple[List[dict], Dict[str, str]]:
    """GET every exporter's /metrics (native HTTP client, which releases the GIL) from up to
    `workers` threads at once, so a refresh over many nodes takes about one node's time even when
    some of them time out; frames keep the order of `urls`. Parse failures are reported, not raised.
    https:// URLs (exporters serving TLS) are verified against `ca_file`, else the system bundle.
    `token`: sent as "Authorization: Bearer <token>" (exporters with http_auth_token_file)."""
    from concurrent.futures import ThreadPoolExecutor

    from .._native import core

    c = core()
    headers = f"Authorization: Bearer {token}\r\n" if token else ""

    def one(u):
        return c.http_request("GET", u, "", headers, timeout_s, ca_file)

    with ThreadPoolExecutor(max_workers=max(1, min(workers, len(urls) or 1))) as pool:
        answers = list(pool.map(one, urls))
    frames, errors = [], {}
    for u, (status, body, err) in zip(urls, answers):
        if status != 200:
            errors[u] = err or f"HTTP {status}"
            continue
        try:
            frames.append(promtext.parse(body.decode("utf-8", "replace")))
        except promtext.PromParseError as e:
            errors[u] = f"malformed exposition: {e}"
    return frames, errors
