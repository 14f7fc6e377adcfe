#!/bin/bash
# Round-4 GPU pass j: the host's KFD census, then the driver-shape bench twice (the process-list
# phase with the not-on-this-GPU cache), then the process-list tests.
set -o pipefail
out=gpurun_out/r4j
mkdir -p $out
timeout -k 5 30 python3 tools/kfd_census.py > $out/census.json 2>&1 || exit 1
cat $out/census.json
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $out/bench$i.json 2> $out/bench$i.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('$out/bench$i.json').read().strip().splitlines()[-1]); print(json.dumps({k: d.get(k) for k in ('scrape_p99_ms','server_scrape_p99_ms','tick_mean_ms','tick_p99_ms','tick_phases_mean_ms','backend_call_us','device_check')}))"
done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "process or tenant or shared or load_is_visible" > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; exit $rc
