#!/bin/bash
# Round-2 GPU call m: the K1 probe moved into the on-device helper (the exporter never loads HIP):
# on-device GPU tests, per-process CPU / RSS in three shapes, a 3-minute footprint.
set -o pipefail
out=gpurun_out/r2m
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_footprint.py tests/test_gpu_coexist.py -m gpu -x -v -s --timeout 200 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -60 $out/pytest_gpu.txt; exit 1; }
grep -E "passed|failed" $out/pytest_gpu.txt | tail -2
for cfg in "--interval 0.1 --pmc --probe" "--interval 1 --probe" "--interval 1 --pmc"; do
  timeout -k 10 120 python -u tools/thread_cpu.py --seconds 10 -- $cfg >> $out/threads.jsonl 2>> $out/threads.err || { tail $out/threads.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$out/threads.jsonl')][-1]; print(d['flags'], 'exporter cpu', d['total_cpu_pct'], 'rss', round(d['rss_mb']), 'children', d['children'])"
done
timeout -k 10 400 python -u tools/footprint.py --seconds 180 > $out/footprint.json 2> $out/footprint.err || { tail $out/footprint.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/footprint.json')); [print(k, v['cpu_millicores'], v['rss_mb_max']) for k, v in d['configs'].items()]"
echo finished
