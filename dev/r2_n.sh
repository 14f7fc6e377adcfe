#!/bin/bash
# Round-2 GPU call n: probe latency through the helper (one-request cycle) vs in-process; full GPU tests.
set -o pipefail
out=gpurun_out/r2n
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/probe_latency_compare.py --seconds 6 > $out/probe_latency.json 2> $out/probe_latency.err || { tail -20 $out/probe_latency.err; exit 1; }
cat $out/probe_latency.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -60 $out/pytest_gpu.txt; exit 1; }
grep -E "passed|failed" $out/pytest_gpu.txt | tail -2
echo finished
