#!/bin/bash
# Round-4 GPU pass b: the runtime cgroup probe (tenant rows), and the idle-reference experiment on
# a pinned CPU set: the same bench on 8 CPUs without and with 8 SCHED_IDLE spinners on those CPUs.
set -o pipefail
out=gpurun_out/r4b
mkdir -p $out
timeout -k 10 120 python -u tools/runtime_cgroup_probe.py $out/runtime > $out/runtime.log 2>&1 || exit 1
echo runtime_ok
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --capacity-s 0 --pin-cpus 8 \
    --out $out/pin8_$i.json > $out/pin8_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --capacity-s 0 --pin-cpus 8 --idle-spinners 8 \
    --out $out/pin8_spin_$i.json > $out/pin8_spin_$i.log 2>&1 || exit 1
  echo round_$i ok
done
# the deployed configs on the hardware: the DaemonSet ConfigMap and each overlay's config through
# the Python-free entry point (--once), sockets / log tree absent on the box
python - $out <<'PY'
import sys, yaml
out = sys.argv[1]
docs = [d for d in yaml.safe_load_all(open("deploy/k8s/gpumon-daemonset.yaml")) if d]
cm = next(d for d in docs if d["kind"] == "ConfigMap")
open(f"{out}/cm_base.yaml", "w").write(cm["data"]["config.yaml"])
for ov in ("pmc", "ondevice", "stress", "nonroot"):
    k = yaml.safe_load(open(f"deploy/k8s/overlays/{ov}/kustomization.yaml"))
    p = next(p for p in k["patches"] if p["target"]["kind"] == "ConfigMap")
    open(f"{out}/cm_{ov}.yaml", "w").write(yaml.safe_load(p["patch"])[0]["value"])
PY
for c in base pmc ondevice stress nonroot; do
  timeout -k 10 90 ./bin/gpumon-exporter --config $out/cm_$c.yaml --once > $out/cm_$c.prom 2> $out/cm_$c.err || exit 1
  echo "cm_$c families=$(grep -c '^# TYPE' $out/cm_$c.prom)"
done
# per-kernel time of the driver-shape bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o r4b -- python3 bench.py --steps 5 --warmup 1 \
  --capacity-s 0 --idle-s 2 > $out/prof.log 2>&1 || exit 1
echo prof_ok
