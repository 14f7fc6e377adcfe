#!/bin/bash
# Round-2 GPU call f: which thread / mapping holds the PMC+probe footprint.
set -o pipefail
out=gpurun_out/r2f
mkdir -p $out
export TMPDIR=/tmp
for cfg in "--interval 0.1" "--interval 0.1 --pmc" "--interval 0.1 --probe" "--interval 0.1 --pmc --pmc-mode window" "--interval 1 --pmc --probe"; do
  timeout -k 10 120 python -u tools/thread_cpu.py --seconds 12 -- $cfg >> $out/threads.jsonl 2>> $out/threads.err || { tail $out/threads.err; exit 1; }
  tail -1 $out/threads.jsonl
done
echo finished
