#!/bin/bash
# Round-4 GPU pass e: why does the 10 Hz loaded scrape p99 (0.5-0.7 ms, server 0.18 ms) sit 10x
# above 1 Hz loaded and 10 Hz idle? One factor at a time, 20 s timed each (4000 scrapes).
set -o pipefail
out=gpurun_out/r4e
mkdir -p $out
run() {  # name, extra args
  local n=$1; shift
  timeout -k 10 150 python -u bench.py --interval 0.1 --steps 200 --warmup 5 --capacity-s 0 --idle-s 0 "$@" \
    --out $out/$n.json > $out/$n.log 2>&1 || exit 1
  echo "$n ok"
}
run base
run noprocs --set processes=false
run nogzip --set gzip=false
run mfma --load mfma
run hbm --load hbm
run seq --sample-threads 0
run noprewarm --prewarm-ms 0
run base2
