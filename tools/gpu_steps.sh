#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that faults,
# aborts, segfaults, times out or is killed (exit >= 124), per the pool's rules.  A plain test
# failure (exit 1) does not stop later steps.  Usage: tools/gpu_steps.sh "<secs>|<cmd>" ...
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  secs="${spec%%|*}"; cmd="${spec#*|}"
  i=$((i+1))
  echo "=== step $i (limit ${secs}s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "=== step $i rc=$rc ($(( $(date +%s) - start ))s)" | tee -a gpurun_out/steps.log
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then
    echo "stopping: step $i ended with rc=$rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
