#!/usr/bin/env python3
"""bench.py JSON lines (tools/scaling_rehearsal.sh -> gpurun_out/scaling/results.jsonl) -> the
markdown table used in profiles/r1_scaling_rehearsal.md."""

import json
import sys


# row order written by tools/scaling_rehearsal.sh
NOTES = [""] * 8 + ["--sample-threads 0 (sequential)", "--no-fast-path (libamd_smi only)", "--probe (K1 each tick)",
                    "idle GPU (no load)"]


def main(path="gpurun_out/scaling/results.jsonl"):
    rows = [json.loads(l) for l in open(path) if l.strip().startswith("{")]
    print("| interval | sampled GPUs | note | samples/s | scrape p50 ms | scrape p99 ms | scrape max ms "
          "| idle scrape p99 ms | tick mean ms | tick p99 ms | overruns | gpu_metrics us | process list us | body KB |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for i, d in enumerate(rows):
        notes = [NOTES[i]] if i < len(NOTES) and NOTES[i] else []
        if "mock" in d.get("data", ""):
            notes.append("MOCK")
        calls = d.get("backend_call_us", {})
        cfg = d.get("config", {})
        print(f"| {cfg.get('interval_s')} s | {d.get('sampled_devices')} | {', '.join(notes)} | {d['value']} "
              f"| {d['scrape_p50_ms']} | {d['scrape_p99_ms']} | {d['scrape_max_ms']} "
              f"| {(d.get('scrape_idle') or {}).get('scrape_p99_ms', '')} | {d['tick_mean_ms']} "
              f"| {d['tick_p99_ms']} | {d['overruns']} | {calls.get('gpu_metrics', '')} "
              f"| {calls.get('process_list', '')} | {d['scrape_body_kb']} |")


if __name__ == "__main__":
    main(*sys.argv[1:])
