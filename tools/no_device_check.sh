#!/bin/bash
# What the default exporter still exports WITHOUT access to /dev/kfd and /dev/dri -- the situation
# of an unprivileged DaemonSet pod (drop `privileged: true`): the device cgroup
# refuses the hostPath device nodes. bin/gpumon-exporter-nodev (`make nodev`) is the exporter with
# every open of /dev/kfd and /dev/dri/* refused with EPERM (csrc/testtools/nodev_interpose.cpp,
# interposed on libamd_smi / libdrm / hsakmt); bin/gpumon-exporter is the reference run. A torch
# tenant keeps a KFD process on the GPU meanwhile, so the process rows are compared too.
# (A user + mount namespace that hides the nodes is not available on the gpurun boxes.)
#
#   tools/no_device_check.sh [OUTDIR]      (on the GPU box; writes OUTDIR/{with_dev,no_dev}.prom, summary.json)
set -o pipefail
out=${1:-gpurun_out/nodev}
mkdir -p "$out"
# a test tool, not part of `make all`: build it on the CPU side first (`make tools`)
[ -x ./bin/gpumon-exporter-nodev ] || { echo "bin/gpumon-exporter-nodev missing: run 'make tools' first" >&2; exit 2; }
ARGS="--backend amdsmi --once --no-pod-resources --no-cri --log-level warn"
python -c "import torch,time; x=torch.randn(8192,8192,device='cuda'); t=time.time()
while time.time()-t<25: y=x@x; torch.cuda.synchronize()" > "$out/tenant.log" 2>&1 &
tenant=$!
sleep 12
timeout -k 5 60 ./bin/gpumon-exporter $ARGS > "$out/with_dev.prom" 2> "$out/with_dev.err"
rc1=$?
timeout -k 5 60 ./bin/gpumon-exporter-nodev $ARGS > "$out/no_dev.prom" 2> "$out/no_dev.err"
rc2=$?
# which device nodes a running default exporter keeps open (complementary evidence)
./bin/gpumon-exporter --backend amdsmi --interval 0.5 --listen 127.0.0.1:0 --no-pod-resources --no-cri \
  --log-level warn > /dev/null 2>&1 &
ex=$!
sleep 4
ls -l /proc/$ex/fd 2>/dev/null | grep -o '/dev/[a-z/A-Z0-9]*' | sort | uniq -c > "$out/open_device_nodes.txt" || true
kill $ex; wait $ex 2>/dev/null
wait $tenant
python - "$out" "$rc1" "$rc2" <<'EOF'
import json, sys
sys.path.insert(0, ".")
from gpumon.export import promtext
out, rc1, rc2 = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
a = promtext.parse(open(f"{out}/with_dev.prom").read())
b = promtext.parse(open(f"{out}/no_dev.prom").read())
count = lambda f: {k: len(v["samples"]) for k, v in f.items()}
ca, cb = count(a), count(b)
res = {"rc_with_dev": rc1, "rc_no_dev": rc2, "families_with_dev": len(ca), "families_no_dev": len(cb),
       "missing_without_dev": sorted(k for k in ca if k not in cb),
       "fewer_samples_without_dev": {k: [ca[k], cb[k]] for k in ca if k in cb and cb[k] < ca[k]},
       "pod_rows": [len(a.get("pod_gpu_used_memory", {}).get("samples", [])),
                    len(b.get("pod_gpu_used_memory", {}).get("samples", []))]}
json.dump(res, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(res))
EOF
