#!/bin/bash
# Same-box A/B of the round-4 HEAD tree (ab/r4, a git worktree of df34618 built in-tree) against
# this tree: the driver's bench command with its defaults, alternated 3 times.
# This tree runs twice per alternation: its default (the shipped binary as a child process) and
# --exporter inprocess (the embedding round 4 measured).
set -e
out=gpurun_out/${1:-ab}
mkdir -p "$out"
for i in 1 2 3; do
  (cd ab/r4 && timeout -k 10 150 python -u bench.py --out "../../$out/r4_$i.json" > "../../$out/r4_$i.log" 2>&1)
  timeout -k 10 150 python -u bench.py --out "$out/child_$i.json" > "$out/child_$i.log" 2>&1
  timeout -k 10 150 python -u bench.py --exporter inprocess --out "$out/inproc_$i.json" > "$out/inproc_$i.log" 2>&1
done
