#!/bin/bash
# Round-2 GPU call l: full GPU tests with the PMC helper, its CPU / RSS, a 3-minute footprint.
set -o pipefail
out=gpurun_out/r2l
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -60 $out/pytest_gpu.txt; exit 1; }
grep -E "coexist:|passed|failed" $out/pytest_gpu.txt | tail -4
for cfg in "--interval 0.1 --pmc --probe" "--interval 1 --pmc"; do
  timeout -k 10 120 python -u tools/thread_cpu.py --seconds 10 -- $cfg >> $out/threads.jsonl 2>> $out/threads.err || { tail $out/threads.err; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$out/threads.jsonl')][-1]; print(d['flags'], 'exporter cpu', d['total_cpu_pct'], 'rss', round(d['rss_mb']), 'children', d['children'])"
done
timeout -k 10 400 python -u tools/footprint.py --seconds 180 > $out/footprint.json 2> $out/footprint.err || { tail $out/footprint.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/footprint.json')); [print(k, v['cpu_millicores'], v['rss_mb_max']) for k, v in d['configs'].items()]"
echo finished
