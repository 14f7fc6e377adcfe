#!/bin/bash
# Run GPU steps one after another on the gpurun box, each under its own time limit, recording
# every exit status in OUT/steps.txt. An ordinary failure (exit 1 or 2: a failed assertion) does
# not stop the session; a time limit (124, 137), an abort (134) or a segfault (139) does -- nothing
# more touches the GPU after those.
#
#   tools/gpu_steps.sh OUT  'name|seconds|command' ...
set -o pipefail
out=$1
shift
mkdir -p "$out"
: > "$out/steps.txt"
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc $(( $(date +%s) - start ))s" | tee -a "$out/steps.txt"
  case $rc in
    0|1|2) ;;
    *) echo "stopping: $name ended with $rc" | tee -a "$out/steps.txt"; exit $rc ;;
  esac
done
exit 0
