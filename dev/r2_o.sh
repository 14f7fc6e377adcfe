#!/bin/bash
# Round-2 GPU call o: bench after gzip-after-publish, with the tick phase split (wake / device calls).
set -o pipefail
out=gpurun_out/r2o
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python -u bench.py --out $out/bench_1hz.json > /dev/null 2> $out/bench_1hz.err || { tail -30 $out/bench_1hz.err; exit 1; }
timeout -k 10 120 python -u bench.py --interval 0.1 --steps 300 --warmup 10 --out $out/bench_10hz.json > /dev/null 2> $out/bench_10hz.err || { tail -30 $out/bench_10hz.err; exit 1; }
timeout -k 10 120 python -u bench.py --replicate 8 --steps 20 --out $out/bench_rep8.json > /dev/null 2> $out/bench_rep8.err || { tail -30 $out/bench_rep8.err; exit 1; }
timeout -k 10 120 python -u bench.py --replicate 8 --interval 0.1 --steps 200 --warmup 10 --out $out/bench_rep8_10hz.json > /dev/null 2> $out/bench_rep8_10hz.err || { tail -30 $out/bench_rep8_10hz.err; exit 1; }
for f in $out/bench_*.json; do python3 -c "
import json; d=json.load(open('$f'))
print('$f', d['sampled_devices'], d['config']['interval_s'], 'scrape p50/p99', d['scrape_p50_ms'], d['scrape_p99_ms'], 'tick mean/p99/max', d['tick_mean_ms'], d['tick_p99_ms'], d['tick_max_ms'], 'over', d['overruns'])
print('  phases', d['tick_phases_mean_ms']); print('  slowest', d['slowest_tick']); print('  calls', d['backend_call_us'], 'load', d['load_tflops'], d['load_tbps'])"; done
echo finished
