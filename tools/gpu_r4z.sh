#!/bin/bash
# Round-4 final GPU pass: full pytest -m gpu, smoke(), the driver-shape bench, and rocprofv3 kernel
# stats of the bench (csv) on the final tree.
set -o pipefail
out=gpurun_out/${R4Z_OUT:-r4z}
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -2 $out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $out/bench.json 2> $out/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print(json.dumps({k: d.get(k) for k in ('value','scrape_p99_ms','server_scrape_p99_ms','tick_mean_ms','tick_p99_ms','overruns','device_check')}))"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/prof -o ${R4Z_OUT:-r4z} -- python3 bench.py --steps 5 --warmup 1 > $out/prof_bench.log 2>&1 || exit 1
find $out/prof -name "*kernel_stats*.csv" | head -3
