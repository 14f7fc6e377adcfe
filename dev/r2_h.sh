#!/bin/bash
# Round-2 GPU call h: HSA env knobs vs the spinning pmc-hsa thread.
set -o pipefail
out=gpurun_out/r2h
mkdir -p $out
export TMPDIR=/tmp
for e in HSA_DISABLE_PC_SAMPLING=1 HSA_ENABLE_MWAITX=0 HSA_SIGNAL_WAIT_ABORT_TIMEOUT=0 HSA_DISCOVER_COPY_AGENTS=0; do
  timeout -k 10 120 python -u tools/thread_cpu.py --seconds 6 --no-load --env $e -- --interval 1 --pmc >> $out/threads.jsonl 2>> $out/threads.err || { tail $out/threads.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$out/threads.jsonl')][-1]; print(d['env'], d['total_cpu_pct'], [(t['name'], t['cpu_pct']) for t in d['top'][:3]])"
done
echo finished
