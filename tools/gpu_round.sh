#!/bin/bash
# GPU validation round: gpu tests -> 1-GPU bench -> rocprofv3 kernel stats of the bench.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
out=gpurun_out/round
mkdir -p $out
export TMPDIR=/tmp
echo "[gpu_round] tests" && \
timeout -k 10 420 python -m pytest tests -m gpu -x -q -s > $out/pytest_gpu.txt 2>&1 && \
echo "[gpu_round] bench" && \
timeout -k 10 180 python bench.py --steps 10 --warmup 2 --out $out/bench.json > $out/bench.log 2>&1 && \
echo "[gpu_round] rocprof" && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/prof -o bench -- python3 bench.py --steps 5 --warmup 1 > $out/rocprof.log 2>&1
rc=$?
echo "[gpu_round] rc=$rc"
tail -5 $out/pytest_gpu.txt
exit $rc
