#!/bin/bash
# Reproduces the round-2 MI355X measurements (profiles/) on one GPU box. Every GPU step runs under
# its own time limit and the first failure ends the script. Results land in $OUT (default
# gpurun_out/validate). Run one step per call, e.g. through gpurun:
#
#   tools/gpu_validate.sh tests        pytest -m gpu (the hardware suite)
#   tools/gpu_validate.sh smoke        __graft_entry__.smoke()
#   tools/gpu_validate.sh bench        the driver's bench command, 1 Hz and 10 Hz, 8 replicas
#   tools/gpu_validate.sh profile      rocprofv3 --kernel-trace --stats over a 5-tick bench
#   tools/gpu_validate.sh tenant       tenant overhead (profiles/r2_tenant_overhead.md)
#   tools/gpu_validate.sh footprint    deployed-shape footprint, SECONDS (default 600)
#   tools/gpu_validate.sh threads      per-thread / per-process CPU of the on-device configurations
#   tools/gpu_validate.sh latency      probe latency (helper vs in-process), per-file read latency
set -o pipefail
OUT=${OUT:-gpurun_out/validate}
mkdir -p "$OUT"
export TMPDIR=/tmp

summary() {  # one bench JSON -> one line
  python3 -c "
import json, sys; d = json.load(open(sys.argv[1]))
print(sys.argv[1], {k: d.get(k) for k in ('value', 'scrape_p50_ms', 'scrape_p99_ms', 'tick_mean_ms', 'tick_p99_ms', 'overruns', 'load_tflops', 'load_tbps')})
print('  idle', d.get('scrape_idle')); print('  phases', d.get('tick_phases_mean_ms'))" "$1"
}

case "$1" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 \
      || { tail -60 "$OUT/pytest_gpu.txt"; exit 1; }
    grep -E "passed|failed" "$OUT/pytest_gpu.txt" | tail -1 ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -30 "$OUT/smoke.txt"; exit 1; }
    tail -1 "$OUT/smoke.txt" ;;
  bench)
    timeout -k 10 150 python -u bench.py --steps 20 --out "$OUT/bench_1hz.json" > /dev/null 2> "$OUT/bench_1hz.err" || { tail -30 "$OUT/bench_1hz.err"; exit 1; }
    timeout -k 10 150 python -u bench.py --interval 0.1 --steps 300 --warmup 10 --out "$OUT/bench_10hz.json" > /dev/null 2> "$OUT/bench_10hz.err" || { tail -30 "$OUT/bench_10hz.err"; exit 1; }
    timeout -k 10 150 python -u bench.py --replicate 8 --steps 20 --out "$OUT/bench_rep8.json" > /dev/null 2> "$OUT/bench_rep8.err" || { tail -30 "$OUT/bench_rep8.err"; exit 1; }
    for f in "$OUT"/bench_*.json; do summary "$f"; done ;;
  profile)
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 bench.py --steps 5 --warmup 1 > "$OUT/prof.log" 2>&1 \
      || { tail -30 "$OUT/prof.log"; exit 1; }
    find "$OUT/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$OUT/kernel_stats.csv"
    head -5 "$OUT/kernel_stats.csv" ;;
  tenant)
    timeout -k 10 300 python -u tools/tenant_overhead.py --reps 3 --window 5 > "$OUT/tenant.json" 2> "$OUT/tenant.err" || { tail -20 "$OUT/tenant.err"; exit 1; }
    tail -3 "$OUT/tenant.err" ;;
  footprint)
    s=${2:-600}
    timeout -k 10 $((s + 120)) python -u tools/footprint.py --seconds "$s" > "$OUT/footprint.json" 2> "$OUT/footprint.err" || { tail "$OUT/footprint.err"; exit 1; }
    python3 -c "import json; d = json.load(open('$OUT/footprint.json')); [print(k, v['cpu_millicores'], v['rss_mb_first'], v['rss_mb_last'], v['rss_mb_max'], v['scrape_errors']) for k, v in d['configs'].items()]" ;;
  threads)
    for cfg in "--interval 0.1 --pmc --probe" "--interval 1 --probe" "--interval 1 --pmc"; do
      timeout -k 10 120 python -u tools/thread_cpu.py --seconds 10 -- $cfg >> "$OUT/threads.jsonl" 2>> "$OUT/threads.err" || { tail "$OUT/threads.err"; exit 1; }
    done
    python3 -c "
import json
for l in open('$OUT/threads.jsonl'):
    d = json.loads(l); print(d['flags'], 'exporter cpu', d['total_cpu_pct'], 'rss', round(d['rss_mb']), 'children', d['children'])" ;;
  latency)
    timeout -k 10 200 python -u tools/probe_latency_compare.py --seconds 6 > "$OUT/probe_latency.json" 2> "$OUT/probe_latency.err" || { tail -20 "$OUT/probe_latency.err"; exit 1; }
    for k in idle mixed concurrent; do
      timeout -k 10 200 python -u tools/sysfs_read_latency.py --kind $k --reads 3000 > "$OUT/lat_$k.json" 2> "$OUT/lat_$k.err" || { tail -20 "$OUT/lat_$k.err"; exit 1; }
    done
    cat "$OUT/probe_latency.err" "$OUT"/lat_*.err ;;
  *)
    sed -n '2,16p' "$0"; exit 2 ;;
esac
