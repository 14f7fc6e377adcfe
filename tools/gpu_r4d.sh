#!/bin/bash
# Round-4 GPU pass d: the SMU's gpu_metrics refresh while idle (doctor) and the 10 Hz bench loaded
# and idle: does a 10 Hz tick ever see a repeated (stale) table, and does stale_hold_s ever withhold
# rates there? Plus the doctor's node report with the on-device check.
set -o pipefail
out=gpurun_out/r4d
mkdir -p $out
timeout -k 10 120 python -u -m gpumon doctor --backend amdsmi --interval 0.1 --ondevice-check --format json \
  > $out/doctor.json 2> $out/doctor.err; rc=$?; echo doctor_rc=$rc
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u bench.py --interval 0.1 --steps 100 --warmup 5 --capacity-s 0 --idle-s 10 \
  --out $out/bench_10hz.json > $out/bench_10hz.log 2>&1 || exit 1
echo bench10_ok
timeout -k 10 200 python -u bench.py --interval 0.1 --steps 100 --warmup 5 --capacity-s 0 --idle-s 0 --load idle \
  --out $out/bench_10hz_idle.json > $out/bench_10hz_idle.log 2>&1 || exit 1
echo bench10_idle_ok
