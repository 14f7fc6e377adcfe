#!/bin/bash
# Round-2 GPU call s: full GPU suite on the current tree, the driver's bench command, kernel stats.
set -o pipefail
out=gpurun_out/r2s
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -60 $out/pytest_gpu.txt; exit 1; }
grep -E "passed|failed" $out/pytest_gpu.txt | tail -1
timeout -k 10 120 python -u bench.py --out $out/bench.json > /dev/null 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print({k: d[k] for k in ('value','vs_baseline','ms_per_step','scrape_p50_ms','scrape_p99_ms','tick_mean_ms','tick_p99_ms','tick_max_ms','overruns','load_tflops','load_tbps')})"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $out/prof -o run -- python3 bench.py --steps 5 --warmup 1 > $out/prof.log 2>&1 || { tail -30 $out/prof.log; exit 1; }
find $out/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $out/kernel_stats.csv
head -5 $out/kernel_stats.csv
echo finished
