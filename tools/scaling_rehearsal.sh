#!/bin/bash
# Sampler/scrape scaling rehearsal on a 1-GPU box: the real MI355X sampled 1/2/4/8 times per tick
# (amdsmi:replicate=R) at 1 Hz and 10 Hz under the synthetic load, plus the probe-kernel variant.
# The official 1/2/4/8-GPU curve is produced by the driver on a full node (bench.py unchanged).
set -o pipefail
out=gpurun_out/scaling
mkdir -p $out
: > $out/results.jsonl
for hz in 1 10; do
  iv=$(python3 -c "print(1.0/$hz)")
  steps=$(( hz == 1 ? 10 : 60 ))
  for r in 1 2 4 8; do
    timeout -k 10 150 python bench.py --steps $steps --warmup 2 --interval $iv --replicate $r \
      --scrape-rate 20 --out $out/b_${hz}hz_r${r}.json > $out/log_${hz}hz_r${r}.txt 2>&1 || exit 1
    cat $out/b_${hz}hz_r${r}.json >> $out/results.jsonl
    echo "done hz=$hz r=$r"
  done
done
timeout -k 10 150 python bench.py --steps 10 --warmup 2 --interval 1.0 --replicate 8 --sample-threads 0 \
  --out $out/b_1hz_r8_seq.json > $out/log_seq.txt 2>&1 && cat $out/b_1hz_r8_seq.json >> $out/results.jsonl
timeout -k 10 150 python bench.py --steps 10 --warmup 2 --interval 1.0 --no-fast-path \
  --out $out/b_1hz_nofast.json > $out/log_nofast.txt 2>&1 && cat $out/b_1hz_nofast.json >> $out/results.jsonl
timeout -k 10 150 python bench.py --steps 10 --warmup 2 --interval 1.0 --probe \
  --out $out/b_1hz_probe.json > $out/log_probe.txt 2>&1 && cat $out/b_1hz_probe.json >> $out/results.jsonl
timeout -k 10 150 python bench.py --steps 10 --warmup 2 --interval 1.0 --load idle \
  --out $out/b_1hz_idle.json > $out/log_idle.txt 2>&1 && cat $out/b_1hz_idle.json >> $out/results.jsonl
echo finished
