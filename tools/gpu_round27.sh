#!/bin/bash
# Every on-device feature at once on MI355X: native exporter at 10 Hz with --pmc --probe and RAS
# every tick, GPU under the mixed K2 load; client-side scrape latency + the exporter's own tick
# histogram / per-call accounting.
set -o pipefail
out=gpurun_out/r27
mkdir -p $out
export TMPDIR=/tmp
python -m gpumon load --kind mixed --seconds 40 > $out/load.json 2> $out/load.err &
lp=$!
sleep 6
timeout -k 10 60 ./bin/gpumon-exporter --backend amdsmi --interval 0.1 --pmc --probe --ras-every 1 \
  --listen 127.0.0.1:9411 --log-level warn > $out/exporter.log 2>&1 &
ep=$!
sleep 8
timeout -k 10 60 python -m gpumon scrape http://127.0.0.1:9411/metrics -n 3000 -c 2 > $out/scrape.json 2>&1
rc=$?
python - <<'PY' > $out/metrics.prom
import urllib.request
print(urllib.request.urlopen("http://127.0.0.1:9411/metrics", timeout=5).read().decode())
PY
kill -TERM $ep
wait $ep
wait $lp
cat $out/scrape.json
grep -E '^gpumon_(sample_duration_seconds_(sum|count)|tick_overruns_total|ticks_total|backend_call_seconds_total|backend_calls_total|pmc_errors_total)|^gpu_(mfma_busy|occupancy|probe_latency|probe_kernel_span|probe_wave_slot_mean|gui_active)' $out/metrics.prom
echo "rc=$rc"
exit $rc
