#!/bin/bash
# The one GPU-session runner: every MI355X measurement behind profiles/ is a named step here.
# Steps run in order, each under its own time limit; the FIRST non-zero exit status (a failed test
# included) ends the session, so nothing more touches the GPU after a failure, a time limit
# (124/137), an abort (134) or a segfault (139). Results land in gpurun_out/<run>/.
#
#   tools/gpu_run.sh RUN STEP [STEP ...]
#   gpurun --timeout 900 -- tools/gpu_run.sh r5a tests smoke bench profile
#
# A STEP is one of the names below, or an ad-hoc 'name|seconds|command' spec.
#   tests       pytest -m gpu (the hardware suite)
#   smoke       __graft_entry__.smoke()
#   bench       the driver's bench command (bench.py --steps 10 --warmup 2)
#   bench10     the stress shape: 10 Hz, 100 timed ticks, gzip scrapes, 1 and 8 sampled devices
#   profile     rocprofv3 --kernel-trace --stats over a 5-tick bench (kernel_stats.csv)
#   cpu8        per-thread exporter CPU at 10 Hz + 10 scrapes/s: mock 8 GPUs, amdsmi x8, x8 sequential,
#               amdsmi x1 (profiles/r5_cpu_8dev.md)
#   cpu8x       the amdsmi shapes again with occupancy sub-sampling / prewarm off (what contends)
#   closure     the runtime image's library closure (deploy/image_closure.py) with the real backend
#               and the PMC overlay; /proc/<pid>/maps checked against it
#   tenant      tenant overhead (profiles/r2_tenant_overhead.md)
#   churn       4-minute process-churn soak at 10 Hz: missed / stale rows, RSS / fds / threads trend
#   soak        10-minute 10 Hz soak under load with 50 scrapes/s: RSS / fds / threads, errors
#   pushsoak    10-minute HTTPS push soak of bin/gpumon-exporter: a TLS sink that closes every 50th
#               connection and fails every 200th request; reconnects, retries, fds / RSS trend
#   tlscost     /metrics over HTTPS vs plain, identity vs gzip: service time and round trip per scrape
#   prodsoak    15 minutes of the hardened deployment at 10 Hz: /metrics over HTTPS with the certificate
#               rotated every minute, HTTPS push to a misbehaving sink, verified gzip scrapes
#   authsoak    prodsoak for 10 minutes with a bearer token on /metrics, replaced (with an overlap)
#               at every certificate rotation
#   mtlssoak    prodsoak for 10 minutes with mutual TLS: the scraper presents a client certificate;
#               each window the probes (no certificate) must get 200 and a certificate-less /metrics 403
#   threads     per-thread / per-process CPU of the on-device configurations
#   latency     probe latency (helper vs in-process), per-file sysfs read latency
#   torchrun1   the torchrun / RCCL branch of bench.py with one rank (--dist)
set -o pipefail
run=${1:?usage: tools/gpu_run.sh RUN STEP...}
shift
OUT=gpurun_out/$run
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/steps.txt"

last_json() {  # the bench's one JSON line, selected keys
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], json.dumps({k: d.get(k) for k in sys.argv[2].split(',') if k in d}))" "$@"
}
BENCH_KEYS=value,scrape_p99_ms,scrape_p99_ci95_ms,server_scrape_p99_ms,tick_mean_ms,tick_p99_ms,overruns,exporter_cpu_millicores,device_check

step_cmd() {  # name -> "seconds|command"
  case "$1" in
    tests) echo "900|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" ;;
    smoke) echo "180|python -u -c 'import __graft_entry__ as g; g.smoke()'" ;;
    bench) echo "300|python -u bench.py --steps 10 --warmup 2 --out $OUT/bench.json && last_json $OUT/bench.json $BENCH_KEYS" ;;
    bench10) echo "600|for r in 1 8; do python -u bench.py --interval 0.1 --steps 100 --warmup 10 --replicate \$r --gzip --capacity-s 0 --out $OUT/hz10_r\$r.json > $OUT/hz10_r\$r.err 2>&1 || exit 1; last_json $OUT/hz10_r\$r.json $BENCH_KEYS,scrape_body_kb; done" ;;
    profile) echo "300|rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 && find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \\; && head -5 $OUT/kernel_stats.csv" ;;
    cpu8) echo "600|python -u tools/cpu_8dev.py --seconds 20 --out $OUT/cpu8.jsonl" ;;
    cpu8x) echo "600|python -u tools/cpu_8dev.py --seconds 20 --only amdsmi1,amdsmi1_occ1,amdsmi8,amdsmi8_occ1,amdsmi8_noprewarm,amdsmi8_seq --out $OUT/cpu8x.jsonl" ;;
    closure) echo "300|python -u deploy/image_closure.py check --backend amdsmi --overlays --out $OUT/closure.json" ;;
    tenant) echo "400|python -u tools/tenant_overhead.py --reps 3 --window 5 > $OUT/tenant.json" ;;
    churn) echo "420|python -u tools/churn_soak.py --minutes 4 > $OUT/churn.json" ;;
    soak) echo "720|python -u tools/soak.py --minutes 10 > $OUT/soak.json" ;;
    pushsoak) echo "720|python -u tools/push_soak.py --minutes 10 > $OUT/pushsoak.json" ;;
    tlscost) echo "300|python -u tools/tls_scrape_cost.py --n 4000 > $OUT/tlscost.jsonl" ;;
    prodsoak) echo "1080|python -u tools/push_soak.py --minutes 15 --serve-tls --rotate-every 60 > $OUT/prodsoak.json" ;;
    authsoak) echo "780|python -u tools/push_soak.py --minutes 10 --serve-tls --rotate-every 60 --token > $OUT/authsoak.json" ;;
    mtlssoak) echo "780|python -u tools/push_soak.py --minutes 10 --serve-tls --rotate-every 60 --mtls > $OUT/mtlssoak.json" ;;
    threads) echo "400|for cfg in '--interval 0.1 --pmc --probe' '--interval 1 --probe' '--interval 1 --pmc'; do python -u tools/thread_cpu.py --seconds 10 -- \$cfg >> $OUT/threads.jsonl || exit 1; done" ;;
    latency) echo "600|python -u tools/probe_latency_compare.py --seconds 6 > $OUT/probe_latency.json && for k in idle mixed concurrent; do python -u tools/sysfs_read_latency.py --kind \$k --reads 3000 > $OUT/lat_\$k.json || exit 1; done" ;;
    torchrun1) echo "300|python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --dist --capacity-s 0 --idle-s 2 --out $OUT/torchrun1.json" ;;
    *'|'*) echo "${1#*|}" ;;
    *) return 1 ;;
  esac
}

export -f last_json
export OUT BENCH_KEYS
for spec in "$@"; do
  name=${spec%%|*}
  if ! sc=$(step_cmd "$spec"); then
    sed -n '2,24p' "$0"
    echo "unknown step: $spec" >&2
    exit 2
  fi
  secs=${sc%%|*}
  cmd=${sc#*|}
  start=$(date +%s)
  timeout -k 10 "$secs" bash -o pipefail -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc $(( $(date +%s) - start ))s" | tee -a "$OUT/steps.txt"
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then
    echo "stopping: step $name exited $rc" | tee -a "$OUT/steps.txt"
    tail -40 "$OUT/$name.log"
    exit $rc
  fi
done
exit 0
