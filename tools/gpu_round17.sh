#!/bin/bash
# On-device plugins on MI355X: GPU suite (native + python PMC/probe paths), smoke(), 1-GPU bench,
# and a rocprofv3 kernel trace of the standalone exporter running its probe plugin.
set -o pipefail
out=gpurun_out/r17
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -40 $out/pytest_gpu.txt; exit 1; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { cat $out/smoke.txt; exit 1; }
cat $out/smoke.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 3 > $out/bench_1hz.json 2> $out/bench_1hz.err || { tail $out/bench_1hz.err; exit 1; }
tail -1 $out/bench_1hz.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof_probe -o probe -- ./bin/gpumon-exporter --backend amdsmi --once --probe --log-level warn > $out/prof_probe.log 2>&1 || { tail -20 $out/prof_probe.log; exit 1; }
find $out/prof_probe -name "*stats*" | head -5
echo finished
