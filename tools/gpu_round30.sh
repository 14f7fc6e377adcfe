#!/bin/bash
set -o pipefail
out=gpurun_out/r30
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pmc.py tests/test_gpu_cli.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest.txt 2>&1 || { tail -40 $out/pytest.txt; exit 1; }
grep -E "PASSED|FAILED" $out/pytest.txt
timeout -k 10 120 python tools/pmc_check.py > $out/pmc_check.json 2> $out/pmc_check.err || { tail $out/pmc_check.err; exit 1; }
python3 -c "import json;d=json.loads(open('$out/pmc_check.json').read().strip().splitlines()[-1]);print({k:d[k] for k in ('idle','mfma','hbm','partial')}, d['mfma_load'])"
echo finished
