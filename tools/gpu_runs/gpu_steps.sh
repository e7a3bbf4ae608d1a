#!/usr/bin/env bash
# Run GPU steps in sequence on the gpurun box; stop at the first step that ends
# in a fault / abort / timeout (rc not in {0,1}).  Each step has its own limit.
#   tools/gpu_runs/gpu_steps.sh "<secs>|<name>|<command>" ...
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"
  name="${rest%%|*}"; cmd="${rest#*|}"
  echo "[gpu_steps] >>> $name ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_steps] <<< $name rc=$rc ($(( $(date +%s) - start )) s)"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "[gpu_steps] stopping: step $name ended with rc=$rc"
    exit $rc
  fi
done
exit 0
