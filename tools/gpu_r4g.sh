#!/bin/bash
# Round-4 GPU pass g: the torchrun / RCCL code path with one rank (--dist): the BDF gather
# (all_gather_object over RCCL), the device pairing and device_check in the distributed branch.
set -o pipefail
out=gpurun_out/r4g
mkdir -p $out
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --dist --capacity-s 0 --idle-s 2 \
  --out $out/torchrun1.json > $out/torchrun1.log 2>&1 || exit 1
echo torchrun1_ok
