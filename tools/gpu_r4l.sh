#!/bin/bash
# Round-4 GPU pass l: A/B of a throwaway process list at prewarm time (GPUMON_PREWARM_PROCS),
# the driver-shape bench alternating A, B, A, B.
set -o pipefail
out=gpurun_out/r4l
mkdir -p $out
for i in 1 2; do
  for v in 0 1; do
    GPUMON_PREWARM_PROCS=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $out/b${i}_$v.json 2> $out/b${i}_$v.err || exit 1
    python3 -c "import json; d=json.loads(open('$out/b${i}_$v.json').read().strip().splitlines()[-1]); ph=d['tick_phases_mean_ms']; print(json.dumps({'run': '$i', 'prewarm_procs': $v, 'tick_mean_ms': d['tick_mean_ms'], 'tick_p99_ms': d['tick_p99_ms'], 't_device': ph['t_device'], 't_procs': ph['t_procs'], 'proc_us': d['backend_call_us'].get('process_list'), 'scrape_p99_ms': d['scrape_p99_ms']}))"
  done
done
