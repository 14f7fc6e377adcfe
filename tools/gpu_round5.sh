#!/bin/bash
# Sampler phases on the GPU timeline: ROCTx ranges (GPUMON_ROCTX=1) + kernel trace while bench.py
# runs at 10 Hz under the mixed MFMA/HBM load. Summaries land in gpurun_out/r5/.
set -o pipefail
out=gpurun_out/r5
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GPUMON_ROCTX=1
timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d $out/prof -o run \
  -- python3 bench.py --steps 30 --warmup 3 --interval 0.1 > $out/bench.json 2> $out/bench.err || exit 1
tail -1 $out/bench.json
find $out/prof -name '*stats.csv' | sort
echo finished
