set -o pipefail
out=gpurun_out/r28
mkdir -p $out
python -m gpumon load --kind mfma --seconds 30 > $out/load.json 2>&1 &
lp=$!
sleep 6
for w in 0.05 0.2; do
  timeout -k 5 60 ./bin/gpumon-exporter --backend amdsmi --once --pmc --pmc-window $w --log-level warn 2>&1 | grep -E "^gpu_(mfma_busy|occupancy|gui)" | sed "s/^/bin w=$w /"
done
timeout -k 5 60 python - <<'PY'
import sys; sys.path.insert(0, ".")
from gpumon.ops.pmc import pmc_module, DEFAULT_COUNTERS, derive
P = pmc_module(); P.init(); a = P.agents()[0]
for w in (0.05, 0.2):
    raw = P.sample(0, DEFAULT_COUNTERS, w)
    print("py w=%s" % w, {k: (v["sum"], v["max"], v["n"]) for k, v in raw.items()}, derive(raw, a))
PY
wait $lp
