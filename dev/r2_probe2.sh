#!/bin/bash
# Round-2 hardware probes: KFD cu_occupancy semantics, continuous PMC reads, concurrent load, tenant overhead.
set -o pipefail
out=gpurun_out/r2b
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/kfd_occupancy_probe.py --kinds mfma,hbm,mixed,concurrent,partial,self-mfma --seconds 2 > $out/kfd_occ.json 2> $out/kfd_occ.err || { tail $out/kfd_occ.err; exit 1; }
cat $out/kfd_occ.err
timeout -k 10 60 python -m gpumon load --kind concurrent --seconds 6 > $out/concurrent.json 2>&1 || { cat $out/concurrent.json; exit 1; }
cat $out/concurrent.json
timeout -k 10 300 python -u tools/pmc_continuous_probe.py > $out/pmc_cont.json 2> $out/pmc_cont.err || { tail -20 $out/pmc_cont.err; exit 1; }
cat $out/pmc_cont.err
timeout -k 10 400 python -u tools/tenant_overhead.py --reps 3 --window 5 > $out/tenant.json 2> $out/tenant.err || { tail -20 $out/tenant.err; exit 1; }
tail -4 $out/tenant.err
echo finished
