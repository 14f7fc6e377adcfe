#!/bin/bash
# Burn shapes after splitting the 16x16x32 burn into its own VGPR-form TU; PMC on the default load;
# GPU tests; 1 Hz bench.
set -o pipefail
out=gpurun_out/${ROUND_TAG:-r10}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/burn_shapes.py > $out/burn_shapes.json 2> $out/burn.err || exit 1
cat $out/burn_shapes.json
timeout -k 10 600 python -m pytest tests -m gpu -x -q -s > $out/pytest_gpu.txt 2>&1; rc=$?
tail -3 $out/pytest_gpu.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $out/bench.json 2> $out/bench.err || exit 1
cat $out/bench.json
echo finished
