#!/bin/bash
# Round-2 first GPU call: gpu tests + smoke + 1 Hz bench + rocprofv3 kernel stats + KFD occupancy probe.
set -o pipefail
out=gpurun_out/r2a
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -40 $out/pytest_gpu.txt; exit 1; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 200 python -u tools/kfd_occupancy_probe.py --kinds mfma,hbm,mixed --seconds 2 > $out/kfd_occ.json 2> $out/kfd_occ.err || { tail $out/kfd_occ.err; exit 1; }
cat $out/kfd_occ.err
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $out/bench_1hz.json 2> $out/bench_1hz.err || { tail $out/bench_1hz.err; exit 1; }
tail -c 1500 $out/bench_1hz.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 5 --warmup 2 > $out/bench_prof.log 2>&1 || { tail $out/bench_prof.log; exit 1; }
find $out/prof -name '*stats*' | head
echo finished
