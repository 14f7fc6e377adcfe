#!/bin/bash
# Re-validation of the restored tree: GPU suite, smoke(), 1-GPU bench at 1 Hz and 10 Hz, rocprofv3 stats.
set -o pipefail
out=gpurun_out/r16
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -30 $out/pytest_gpu.txt; exit 1; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { cat $out/smoke.txt; exit 1; }
cat $out/smoke.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $out/bench_1hz.json 2> $out/bench_1hz.err || { tail $out/bench_1hz.err; exit 1; }
tail -1 $out/bench_1hz.json
timeout -k 10 300 python bench.py --steps 300 --warmup 10 --interval 0.1 > $out/bench_10hz.json 2> $out/bench_10hz.err || { tail $out/bench_10hz.err; exit 1; }
tail -1 $out/bench_10hz.json
echo finished
