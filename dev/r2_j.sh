#!/bin/bash
set -o pipefail
out=gpurun_out/r2j
mkdir -p $out
export TMPDIR=/tmp
for e in GPUMON_PMC_DEBUG_INIT=no-contexts GPUMON_PMC_DEBUG_INIT=no-service; do
  timeout -k 10 120 python -u tools/thread_cpu.py --seconds 5 --no-load --env $e -- --interval 1 --pmc >> $out/threads.jsonl 2>> $out/threads.err || { tail $out/threads.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$out/threads.jsonl')][-1]; print(d['env'], d['total_cpu_pct'], [(t['name'], t['cpu_pct']) for t in d['top'][:3]])"
done
echo finished
