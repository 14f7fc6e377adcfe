#!/bin/bash
# Round-2 GPU call g: which runtime thread spins with --pmc.
set -o pipefail
out=gpurun_out/r2g
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/thread_cpu.py --seconds 8 -- --interval 1 --pmc >> $out/threads.jsonl 2>> $out/threads.err || { tail $out/threads.err; exit 1; }
timeout -k 10 120 python -u tools/thread_cpu.py --seconds 8 --env HSA_ENABLE_INTERRUPT=1 -- --interval 1 --pmc >> $out/threads.jsonl 2>> $out/threads.err || { tail $out/threads.err; exit 1; }
timeout -k 10 120 python -u tools/thread_cpu.py --seconds 8 --no-load -- --interval 1 --pmc >> $out/threads.jsonl 2>> $out/threads.err || { tail $out/threads.err; exit 1; }
cat $out/threads.jsonl
echo finished
