#!/bin/bash
# Round-2 GPU call e: benches with async RAS, then the 10-minute deployed-shape footprint run.
set -o pipefail
out=gpurun_out/r2e
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 30 --warmup 3 > $out/bench_1hz.json 2> $out/bench_1hz.err || { tail $out/bench_1hz.err; exit 1; }
timeout -k 10 300 python bench.py --steps 300 --warmup 10 --interval 0.1 > $out/bench_10hz.json 2> $out/bench_10hz.err || { tail $out/bench_10hz.err; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_1hz", "bench_10hz"):
    d = json.loads(open(f"gpurun_out/r2e/{f}.json").read().strip().splitlines()[-1])
    print(f, {k: d[k] for k in ("scrape_p50_ms", "scrape_p99_ms", "tick_mean_ms", "tick_p99_ms", "tick_max_ms", "overruns", "slowest_tick")})
PY
timeout -k 10 800 python -u tools/footprint.py --seconds 600 > $out/footprint.json 2> $out/footprint.err || { tail $out/footprint.err; exit 1; }
tail -3 $out/footprint.err
python3 -c "import json; d=json.load(open('$out/footprint.json')); [print(k, v) for k, v in d['configs'].items()]"
echo finished
