#!/bin/bash
# Round-4 GPU pass c: the full GPU suite on the current tree (probe paired by PCI address, RT HTTP
# loops, frozen-table hold), then the driver's smoke().
set -o pipefail
out=gpurun_out/r4c
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo pytest_rc=$rc
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
tail -1 $out/smoke.log
