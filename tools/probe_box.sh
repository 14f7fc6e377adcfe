#!/bin/bash
# One-shot environment probe for the GPU box: what amdsmi exposes, permissions, counters.
out=gpurun_out/probe
mkdir -p $out
{
  echo "== id"; id; uname -a; nproc
  echo "== devices"; ls -la /dev/kfd /dev/dri 2>&1
  echo "== perf_event_paranoid"; cat /proc/sys/kernel/perf_event_paranoid 2>&1
  echo "== cgroup self"; cat /proc/self/cgroup
  echo "== env HIP"; env | grep -i -E "HIP|ROCR|HSA|GPU|CUDA" 
} > $out/env.txt 2>&1
timeout -k 10 60 amd-smi static > $out/amdsmi_static.txt 2>&1
timeout -k 10 60 amd-smi metric > $out/amdsmi_metric.txt 2>&1
timeout -k 10 60 amd-smi list > $out/amdsmi_list.txt 2>&1
timeout -k 10 60 amd-smi process > $out/amdsmi_process.txt 2>&1
timeout -k 10 60 amd-smi xgmi > $out/amdsmi_xgmi.txt 2>&1
timeout -k 10 60 amd-smi partition > $out/amdsmi_partition.txt 2>&1
timeout -k 10 60 python3 tools/probe_amdsmi.py > $out/py_amdsmi.txt 2>&1
timeout -k 10 120 rocprofv3 -L > $out/rocprof_L.txt 2>&1
echo done
