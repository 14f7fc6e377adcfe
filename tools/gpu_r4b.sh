#!/bin/bash
# Round-4 GPU pass b: the runtime cgroup probe (tenant rows), and the idle-reference experiment on
# a pinned CPU set: the same bench on 8 CPUs without and with 8 SCHED_IDLE spinners on those CPUs.
set -o pipefail
out=gpurun_out/r4b
mkdir -p $out
timeout -k 10 120 python -u tools/runtime_cgroup_probe.py $out/runtime > $out/runtime.log 2>&1 || exit 1
echo runtime_ok
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --capacity-s 0 --pin-cpus 8 \
    --out $out/pin8_$i.json > $out/pin8_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --capacity-s 0 --pin-cpus 8 --idle-spinners 8 \
    --out $out/pin8_spin_$i.json > $out/pin8_spin_$i.log 2>&1 || exit 1
  echo round_$i ok
done
