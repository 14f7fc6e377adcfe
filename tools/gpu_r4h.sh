#!/bin/bash
# Round-4 GPU pass h: the full GPU suite on the tree with the process-list hold and the bounded
# HTTP request bodies, the driver's smoke(), then the driver-shape bench.
set -o pipefail
out=gpurun_out/r4h
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 $out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
tail -1 $out/smoke.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $out/bench.json 2> $out/bench.err || exit 1
tail -1 $out/bench.json | cut -c1-400
