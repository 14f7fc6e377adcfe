#!/bin/bash
# Round 2 on GPU: all gpu tests, PMC dims, rocprofv3 --pmc cross-check of the burn kernel.
set -o pipefail
out=gpurun_out/r2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests -m gpu -x -q -s > $out/pytest_gpu.txt 2>&1; rc=$?
tail -3 $out/pytest_gpu.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 60 python3 -c "
import gpumon._pmc as P; P.init()
for c in ['SQ_VALU_MFMA_BUSY_CYCLES','GRBM_GUI_ACTIVE','SQ_WAVE_CYCLES','SQ_WAVES','SQ_BUSY_CYCLES','SQ_INSTS_VALU_MFMA_MOPS_BF16']:
    try: print(c, P.counter_dimensions(0, c))
    except Exception as e: print(c, 'ERR', e)
" > $out/pmc_dims.txt 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $out/pmc_prof -o burn -- python3 tools/burn_once.py 10 > $out/rocprof_pmc.log 2>&1
echo "rocprof rc=$?"
