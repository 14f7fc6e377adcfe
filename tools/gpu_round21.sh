#!/bin/bash
# RAS counters + native-probe smoke on MI355X: full GPU suite, smoke(), RAS timing.
set -o pipefail
out=gpurun_out/r21
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -40 $out/pytest_gpu.txt; exit 1; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { cat $out/smoke.txt; exit 1; }
cat $out/smoke.txt
timeout -k 10 60 ./bin/gpumon-exporter --backend amdsmi --once --log-level warn > $out/once.prom 2>&1 || { tail $out/once.prom; exit 1; }
grep -E "^gpu_(ecc|ras|retired)|call=\"ras\"" $out/once.prom | head -40
echo finished
