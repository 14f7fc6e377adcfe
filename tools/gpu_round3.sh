#!/bin/bash
set -o pipefail
out=gpurun_out/r3
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > $out/pytest_gpu.txt 2>&1; rc=$?
tail -3 $out/pytest_gpu.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/kernel_bench.py > $out/kernel_bench.json 2> $out/kernel_bench.err || exit 1
timeout -k 10 120 python3 tools/pmc_check.py > $out/pmc_check.json 2> $out/pmc_check.err || exit 1
echo finished
