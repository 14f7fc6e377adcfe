#!/bin/bash
# Round-2 GPU call r: per-file read latency of the tick path under idle / mixed / concurrent loads.
set -o pipefail
out=gpurun_out/r2r
mkdir -p $out
export TMPDIR=/tmp
for k in idle mixed concurrent; do

  timeout -k 10 200 python -u tools/sysfs_read_latency.py --kind $k --reads 3000 > $out/lat_$k.json 2> $out/lat_$k.err || { tail -20 $out/lat_$k.err; exit 1; }
  echo "== $k"; cat $out/lat_$k.err
done
echo finished
