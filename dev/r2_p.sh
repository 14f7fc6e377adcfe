#!/bin/bash
# Round-2 GPU call p: 10-minute footprint soak with the probe in the helper; tenant overhead re-run.
set -o pipefail
out=gpurun_out/r2p
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/tenant_overhead.py --reps 3 --window 5 > $out/tenant.json 2> $out/tenant.err || { tail -20 $out/tenant.err; exit 1; }
tail -3 $out/tenant.err
timeout -k 10 760 python -u tools/footprint.py --seconds 600 > $out/footprint.json 2> $out/footprint.err || { tail $out/footprint.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/footprint.json')); [print(k, v['cpu_millicores'], v['rss_mb_first'], v['rss_mb_last'], v['rss_mb_max'], v['scrapes'], v['scrape_errors'], v['scrape_ms_max']) for k, v in d['configs'].items()]"
echo finished
