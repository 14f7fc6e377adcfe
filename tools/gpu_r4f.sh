#!/bin/bash
# Round-4 GPU pass f: the 10 Hz loaded scrape tail, A/B of the synthetic load's host wait: HIP's
# default (spin-polling) vs blocking-sync completion events, interleaved x3; the load's
# throughput is in each line (load_tflops / load_tbps).
set -o pipefail
out=gpurun_out/r4f
mkdir -p $out
run() {  # name, env
  local n=$1; shift
  env "$@" timeout -k 10 150 python -u bench.py --interval 0.1 --steps 200 --warmup 5 --capacity-s 0 --idle-s 0 \
    --out $out/$n.json > $out/$n.log 2>&1 || exit 1
  echo "$n ok"
}
for i in 1 2 3; do
  run spin_$i GPUMON_LOAD_SYNC=spin
  run block_$i GPUMON_LOAD_SYNC=blocking
done
