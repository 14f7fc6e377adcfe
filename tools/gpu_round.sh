#!/bin/bash
# The round-end checks on one GPU box, each step under its own time limit, stopping at the first
# failure: the GPU test suite, smoke(), and the driver's bench command.
set -e
out=gpurun_out/${1:-round}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rP --timeout 120 --timeout-method thread > "$out/pytest_gpu.log" 2>&1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
timeout -k 10 180 python -u bench.py --out "$out/bench.json" > "$out/bench.log" 2>&1
