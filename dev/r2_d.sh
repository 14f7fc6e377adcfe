#!/bin/bash
# Round-2 GPU call d: full gpu tests (continuous PMC, coexistence, tenant overhead), benches.
set -o pipefail
out=gpurun_out/r2d
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -60 $out/pytest_gpu.txt; exit 1; }
grep -E "coexist:|passed|failed" $out/pytest_gpu.txt | tail -5
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $out/bench_1hz.json 2> $out/bench_1hz.err || { tail $out/bench_1hz.err; exit 1; }
tail -c 1500 $out/bench_1hz.json
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --load concurrent > $out/bench_conc.json 2> $out/bench_conc.err || { tail $out/bench_conc.err; exit 1; }
python3 -c "
import json; b=json.loads(open('$out/bench_conc.json').read().strip().splitlines()[-1]); print({k:b[k] for k in ('load_tflops','load_tbps','load_per_gpu','proc_rows')})"
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --interval 0.1 > $out/bench_10hz.json 2> $out/bench_10hz.err || { tail $out/bench_10hz.err; exit 1; }
echo finished
