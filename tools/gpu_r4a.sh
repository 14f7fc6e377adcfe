#!/bin/bash
# Round-4 GPU pass: GPU tests, the driver-shape bench, the runtime cgroup probe, the bench with
# SCHED_IDLE spinners during the idle reference (wake-from-idle check). Stops at any crash/timeout.
set -o pipefail
out=gpurun_out/r4a
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --out $out/bench.json > $out/bench.log 2>&1 || exit 1
echo bench_ok
timeout -k 10 120 python -u tools/runtime_cgroup_probe.py $out/runtime > $out/runtime.log 2>&1 || exit 1
echo runtime_ok
timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --idle-spinners 16 --capacity-s 0 \
  --out $out/bench_spin.json > $out/bench_spin.log 2>&1 || exit 1
echo spin_ok
timeout -k 10 120 python -u tools/helper_memory.py -- --pmc > $out/helpermem_pmc.json 2> $out/helpermem_pmc.err || exit 1
echo helpermem_ok
timeout -k 10 400 python -u tools/scrape_contention.py --seconds 6 --rounds 2 --hogs 16 --spinners 16 --flood-s 4 \
  > $out/scrape_contention.json 2> $out/scrape_contention.err || exit 1
echo contention_ok
