#!/bin/bash
set -o pipefail
out=gpurun_out/r2k
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 150 python -u tools/pmc_stop_probe.py > $out/stop.json 2> $out/stop.err || { tail $out/stop.err; exit 1; }
cat $out/stop.err
echo finished
