#!/bin/bash
set -o pipefail
out=gpurun_out/r2i
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/thread_cpu.py --seconds 6 --no-load -- --interval 1 --pmc > $out/threads.jsonl 2> $out/threads.err || { tail $out/threads.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$out/threads.jsonl').read()); print(d['total_cpu_pct']); [print(t) for t in d['top']]"
echo finished
