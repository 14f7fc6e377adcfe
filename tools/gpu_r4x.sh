#!/bin/bash
# Round-4 pass x: the 8-sampled-device rehearsal (the one GPU sampled 8 times) on the final tree,
# identity and gzip scrapes, 20 timed ticks each (round 3's r3g shape).
set -o pipefail
out=gpurun_out/r4x
mkdir -p $out
for mode in identity gzip; do
  extra=""; [ $mode = gzip ] && extra="--gzip"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 2 --replicate 8 $extra > $out/r8_$mode.json 2> $out/r8_$mode.err || exit 1
  python3 -c "import json; d=json.loads(open('$out/r8_$mode.json').read().strip().splitlines()[-1]); print(json.dumps({'mode': '$mode', **{k: d.get(k) for k in ('scrape_body_kb','scrapes','scrape_p50_ms','scrape_p99_ms','scrape_p99_ci95_ms','server_scrape_p99_ms','tick_mean_ms','tick_p99_ms','overruns','tick_phases_mean_ms')}}))"
done
