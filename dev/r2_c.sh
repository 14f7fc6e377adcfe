#!/bin/bash
# Round-2 GPU call c: gpu tests, benches (1 Hz mixed, concurrent), rocprof csv stats, PMC probe v2, tenant overhead.
set -o pipefail
out=gpurun_out/r2c
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -40 $out/pytest_gpu.txt; exit 1; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $out/bench_1hz.json 2> $out/bench_1hz.err || { tail $out/bench_1hz.err; exit 1; }
tail -c 2500 $out/bench_1hz.json
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --load concurrent > $out/bench_conc.json 2> $out/bench_conc.err || { tail $out/bench_conc.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/prof -o run -- python3 bench.py --steps 5 --warmup 2 > $out/bench_prof.log 2>&1 || { tail $out/bench_prof.log; exit 1; }
find $out/prof -name '*stats*'
timeout -k 10 300 python -u tools/pmc_continuous_probe.py > $out/pmc_cont.json 2> $out/pmc_cont.err || { tail -20 $out/pmc_cont.err; exit 1; }
cat $out/pmc_cont.err
timeout -k 10 400 python -u tools/tenant_overhead.py --reps 3 --window 5 > $out/tenant.json 2> $out/tenant.err || { tail -20 $out/tenant.err; exit 1; }
tail -4 $out/tenant.err
echo finished
