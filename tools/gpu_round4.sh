#!/bin/bash
# rocm_smi fallback on hardware + full GPU test tier + 1-GPU bench.
set -o pipefail
out=gpurun_out/${ROUND_TAG:-r4}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > $out/pytest_gpu.txt 2>&1; rc=$?
tail -3 $out/pytest_gpu.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $out/bench.json 2> $out/bench.err || exit 1
cat $out/bench.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --backend rocm_smi > $out/bench_rsmi.json 2> $out/bench_rsmi.err || exit 1
cat $out/bench_rsmi.json
echo finished
