#!/bin/bash
# Round-2 GPU call v: 17-minute soak of the four deployed shapes (footprint tool) next to a load.
set -o pipefail
out=gpurun_out/r2v
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1120 python -u tools/footprint.py --seconds 1000 > $out/footprint.json 2> $out/footprint.err || { tail $out/footprint.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/footprint.json')); [print(k, v['cpu_millicores'], v['rss_mb_first'], v['rss_mb_last'], v['rss_mb_max'], v['scrapes'], v['scrape_errors'], v['scrape_ms_max']) for k, v in d['configs'].items()]"
echo finished
