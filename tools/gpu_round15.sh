#!/bin/bash
set -o pipefail
out=gpurun_out/r15
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > $out/pytest_gpu.txt 2>&1; rc=$?
tail -3 $out/pytest_gpu.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 tools/soak.py --minutes 12 --interval 0.1 --scrape-rate 50 > $out/soak.jsonl 2> $out/soak.err || exit 1
tail -1 $out/soak.jsonl
echo finished
