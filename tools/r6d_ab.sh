set -e
mkdir -p gpurun_out/r6d
B="python -u bench.py --capacity-s 0 --idle-s 5"
for i in 1 2; do
  timeout -k 10 120 $B --out gpurun_out/r6d/child_$i.json > gpurun_out/r6d/child_$i.log 2>&1
  timeout -k 10 120 $B --exporter inprocess --out gpurun_out/r6d/inproc_$i.json > gpurun_out/r6d/inproc_$i.log 2>&1
done
timeout -k 10 120 $B --pin-cpus 4 --out gpurun_out/r6d/child_pin4.json > gpurun_out/r6d/child_pin4.log 2>&1
GPUMON_LOAD_SYNC=blocking timeout -k 10 120 $B --out gpurun_out/r6d/child_blocking.json > gpurun_out/r6d/child_blocking.log 2>&1
nproc > gpurun_out/r6d/nproc.txt; cat /proc/self/status | grep -i cpus_allowed_list >> gpurun_out/r6d/nproc.txt
