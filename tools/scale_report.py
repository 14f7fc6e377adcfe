#!/usr/bin/env python3
"""Read bench lines at several GPU counts (the driver's SCALE record, or bench.py --out files) and
print the table the 8-GPU questions need: per N the whole-node rate and its
scaling efficiency, scrape / tick tails, the exporter's CPU, each sampled device's call times
(one SMU per GPU: do the eight stay at the 1-GPU value?), workload rows per GPU against ranks
(peer contexts hidden?), the hidden contexts by reason, every rank's world size, and the xGMI
cross-check (exporter per-link rates against the all-reduce's expectation, link -> BDF map).

    python tools/scale_report.py SCALE_r06.json            # a JSON list / {"runs": [...]} / JSON lines
    python tools/scale_report.py n1.json n2.json n4.json n8.json
"""

from __future__ import annotations

import json
import sys
from typing import Any, Dict, List


def _lines(path: str) -> List[Dict[str, Any]]:
    text = open(path, encoding="utf-8").read().strip()
    try:
        doc = json.loads(text)
    except ValueError:
        return [json.loads(l) for l in text.splitlines() if l.strip().startswith("{")]
    if isinstance(doc, list):
        return [d for d in doc if isinstance(d, dict)]
    for key in ("runs", "results", "lines"):
        if isinstance(doc.get(key), list):
            return [d.get("line", d) if isinstance(d, dict) else d for d in doc[key]]
    if isinstance(doc, dict) and "metric" in doc:
        return [doc]
    # {"1": {...}, "8": {...}} or {"n1": {...}}
    return [v for v in doc.values() if isinstance(v, dict) and "metric" in v]


def _fmt(v, nd=3):
    if v is None:
        return "-"
    if isinstance(v, float):
        return f"{v:.{nd}f}"
    return str(v)


def rows(lines: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    lines = sorted((l for l in lines if "n_gpus" in l), key=lambda l: l["n_gpus"])
    base = next((l for l in lines if l["n_gpus"] == 1), None)
    out = []
    for l in lines:
        n = l["n_gpus"]
        per_gpu = l["value"] / n if n else None
        eff = (l["value"] / (n * base["value"])) if base and base.get("value") else None
        dev = l.get("per_device_tick_ms") or []
        tdev = [d.get("t_device_mean_ms") for d in dev if d.get("t_device_mean_ms") is not None]
        gpu_rows = [r.get("rows") for r in (l.get("per_gpu_rows") or [])]
        ranks = l.get("ranks") or []
        x = l.get("xgmi") or {}
        lm = x.get("link_map") or {}
        out.append({
            "n": n, "value": l.get("value"), "per_gpu": per_gpu, "efficiency": eff,
            "p99_ms": l.get("scrape_p99_ms"), "server_p99_ms": l.get("server_scrape_p99_ms"),
            "tick_mean_ms": l.get("tick_mean_ms"), "tick_p99_ms": l.get("tick_p99_ms"),
            "overruns": l.get("overruns"), "stale": l.get("stale_samples"),
            "cpu_mc": l.get("exporter_cpu_millicores"),
            "t_device_ms": (min(tdev), max(tdev)) if tdev else None,
            "rows_per_gpu": gpu_rows, "ranks": len(ranks),
            "world_sizes": sorted({r.get("world_size") for r in ranks}) if ranks else [],
            "hidden": l.get("hidden_context_reasons"), "peer_hidden": l.get("hidden_peer_contexts"),
            "xgmi_vs_expected": x.get("exporter_vs_expected"), "xgmi_rx_vs_expected": x.get("exporter_rx_vs_expected"),
            "busbw_GBps": x.get("allreduce_busbw_GBps"),
            # peers whose moving link maps to their BDF / peers, and rates within 15 % (bench.py _link_map_check)
            "link_map": (lm.get("error") or f"{lm.get('peers_matched', '?')}/{lm.get('peers', '?')} peers, "
                         f"{lm.get('rates_within_15pct', '?')} rates") if isinstance(lm, dict) and lm else None,
            "device_check": (l.get("device_check") or {}).get("ok"),
            "exporter": l.get("exporter"), "data": l.get("data"),
        })
    return out


def render(rs: List[Dict[str, Any]]) -> str:
    hdr = ("| N | samples/s | per GPU | efficiency | client p99 ms | server p99 ms | tick mean / p99 ms | overruns "
           "| exporter CPU mc | t_device ms (min-max over GPUs) | workload rows per GPU | ranks (world size) "
           "| hidden contexts | xGMI tx / rx vs expected | bus BW GB/s | link map | device check |")
    lines = [hdr, "|" + "---|" * (hdr.count("|") - 1)]
    for r in rs:
        td = "-" if not r["t_device_ms"] else f"{r['t_device_ms'][0]:.3f}-{r['t_device_ms'][1]:.3f}"
        lines.append(
            f"| {r['n']} | {_fmt(r['value'], 4)} | {_fmt(r['per_gpu'], 4)} | {_fmt(r['efficiency'], 3)} "
            f"| {_fmt(r['p99_ms'])} | {_fmt(r['server_p99_ms'])} | {_fmt(r['tick_mean_ms'])} / {_fmt(r['tick_p99_ms'])} "
            f"| {_fmt(r['overruns'])} | {_fmt(r['cpu_mc'], 1)} | {td} | {r['rows_per_gpu'] or '-'} "
            f"| {r['ranks']} ({','.join(map(str, r['world_sizes'])) or '-'}) | {r['hidden'] or '-'} "
            f"| {_fmt(r['xgmi_vs_expected'])} / {_fmt(r['xgmi_rx_vs_expected'])} | {_fmt(r['busbw_GBps'], 1)} "
            f"| {r['link_map'] or '-'} | {_fmt(r['device_check'])} |")
    notes = []
    for r in rs:
        if r["rows_per_gpu"] and r["ranks"] > 1 and any(x != r["ranks"] // r["n"] for x in r["rows_per_gpu"]):
            notes.append(f"N={r['n']}: workload rows per GPU {r['rows_per_gpu']} differ from ranks per GPU "
                         f"({r['ranks'] // r['n']}): peer contexts not all hidden, or a rank missing")
        if r["world_sizes"] and r["world_sizes"] != [r["ranks"]]:
            notes.append(f"N={r['n']}: ranks report world sizes {r['world_sizes']}")
        if r["efficiency"] is not None and r["efficiency"] < 0.95:
            notes.append(f"N={r['n']}: scaling efficiency {r['efficiency']:.3f} < 0.95")
    return "\n".join(lines + ([""] + [f"- {n}" for n in notes] if notes else []))


def main(argv: List[str]) -> int:
    if not argv:
        print(__doc__, file=sys.stderr)
        return 2
    lines: List[Dict[str, Any]] = []
    for p in argv:
        lines.extend(_lines(p))
    print(render(rows(lines)))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
