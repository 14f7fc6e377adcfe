#!/bin/bash
# Full GPU suite + smoke + 1 Hz / 10 Hz bench on the current tree.
set -o pipefail
out=gpurun_out/${GPUMON_ROUND_DIR:-r32}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -40 $out/pytest_gpu.txt; exit 1; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { cat $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $out/bench_1hz.json 2> $out/bench_1hz.err || { tail $out/bench_1hz.err; exit 1; }
timeout -k 10 300 python bench.py --steps 300 --warmup 10 --interval 0.1 > $out/bench_10hz.json 2> $out/bench_10hz.err || { tail $out/bench_10hz.err; exit 1; }
GPUMON_ROUND_DIR=${GPUMON_ROUND_DIR:-r32} python3 - <<'PY'
import json, os
for f in ("bench_1hz", "bench_10hz"):
    d = json.loads(open(f"gpurun_out/{os.environ.get('GPUMON_ROUND_DIR', 'r32')}/{f}.json").read().strip().splitlines()[-1])
    print(f, {k: d[k] for k in ("value", "vs_baseline", "scrape_p50_ms", "scrape_p99_ms", "tick_mean_ms", "tick_p99_ms", "overruns", "load_tflops", "load_tbps")})
PY
echo finished
