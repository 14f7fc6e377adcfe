#!/bin/bash
# Round-4 pass w: the stress shape (10 Hz) with 8 sampled devices, gzip scrapes, and 1 device for
# reference; 100 timed ticks each.
set -o pipefail
out=gpurun_out/r4w
mkdir -p $out
for r in 1 8; do
  timeout -k 10 300 python -u bench.py --interval 0.1 --steps 100 --warmup 10 --replicate $r --gzip > $out/hz10_r$r.json 2> $out/hz10_r$r.err || exit 1
  python3 -c "import json; d=json.loads(open('$out/hz10_r$r.json').read().strip().splitlines()[-1]); print(json.dumps({'replicate': $r, **{k: d.get(k) for k in ('value','scrape_body_kb','scrapes','scrape_p99_ms','scrape_p99_ci95_ms','server_scrape_p99_ms','tick_mean_ms','tick_p99_ms','overruns','exporter_cpu_millicores')}}))"
done
