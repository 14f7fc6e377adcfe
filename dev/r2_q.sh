#!/bin/bash
# Round-2 GPU call q: smoke with the probe through the helper, bench with the fd-table cache,
# scrape-rate sensitivity of the client-side p99.
set -o pipefail
out=gpurun_out/r2q
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -30 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
for r in 20 100 20 100; do
  timeout -k 10 120 python -u bench.py --steps 20 --scrape-rate $r --out $out/bench_r$r.json > /dev/null 2> $out/bench_r$r.err || { tail -30 $out/bench_r$r.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/bench_r$r.json'))
print('rate $r', 'n', d['scrapes'], 'p50/p99/max', d['scrape_p50_ms'], d['scrape_p99_ms'], d['scrape_max_ms'], 'srv p99', d['server_scrape_p99_ms_last4096'], 'tick', d['tick_mean_ms'], d['tick_p99_ms'], d['tick_phases_mean_ms'])"
done
echo finished
