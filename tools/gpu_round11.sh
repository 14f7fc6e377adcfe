#!/bin/bash
# Per-process rows under load, native binary one-shot with the fast path, CLI smoke.
set -o pipefail
out=gpurun_out/r11
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 > $out/bench.json 2> $out/bench.err || exit 1
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['proc_rows'], d['backend_call_us'], d['tick_mean_ms'])"
timeout -k 10 60 ./bin/gpumon-exporter --once > $out/native_once.prom 2> $out/native_once.err || exit 1
grep -c . $out/native_once.prom
grep -E "^gpumon_fast_path_devices|^node_gpu_gpu_util|^gpu_power_watts" $out/native_once.prom
timeout -k 10 120 python3 -m gpumon once --format json > $out/once.json 2> $out/once.err || exit 1
timeout -k 10 60 python3 -m gpumon xgmi > $out/xgmi.json 2>&1 || exit 1
cat $out/xgmi.json
echo finished
