#!/bin/bash
# Round-4 pass v: exporter CPU at 10 Hz with 8 sampled devices against occ_samples (between-tick
# KFD occupancy reads per tick): 20 (the default) vs 4 vs 2.
set -o pipefail
out=gpurun_out/r4v
mkdir -p $out
for occ in 20 4 2; do
  timeout -k 10 300 python -u bench.py --interval 0.1 --steps 100 --warmup 10 --replicate 8 --gzip --set occ_samples=$occ > $out/occ$occ.json 2> $out/occ$occ.err || exit 1
  python3 -c "import json; d=json.loads(open('$out/occ$occ.json').read().strip().splitlines()[-1]); print(json.dumps({'occ_samples': $occ, **{k: d.get(k) for k in ('value','scrape_p99_ms','tick_mean_ms','tick_p99_ms','overruns','exporter_cpu_millicores','occupancy_reads')}}))"
done
