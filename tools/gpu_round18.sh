#!/bin/bash
# Probe publication rework (hierarchical arrival): probe/plugin GPU tests + rocprofv3 kernel trace
# of the standalone exporter's probe plugin, idle and under the MFMA burn.
set -o pipefail
out=gpurun_out/r18
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_device.py tests/test_gpu_cli.py -m gpu -x -v --timeout 200 --timeout-method thread -k "probe or cli or smoke or native or once" > $out/pytest_gpu.txt 2>&1 || { tail -40 $out/pytest_gpu.txt; exit 1; }
grep -E "PASSED|FAILED" $out/pytest_gpu.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof_idle -o probe -- ./bin/gpumon-exporter --backend amdsmi --once --probe --log-level warn > $out/prof_idle.log 2>&1 || { tail -20 $out/prof_idle.log; exit 1; }
grep -E "^gpu_probe_(latency|kernel_span|stale|unique)" $out/prof_idle.log
python -m gpumon load --kind mfma --seconds 14 > $out/load.log 2>&1 &
lp=$!
sleep 6
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof_load -o probe -- ./bin/gpumon-exporter --backend amdsmi --once --probe --log-level warn > $out/prof_load.log 2>&1 || { tail -20 $out/prof_load.log; wait $lp; exit 1; }
wait $lp
grep -E "^gpu_probe_(latency|kernel_span|stale|unique)" $out/prof_load.log
echo finished
