#!/usr/bin/env bash
# counters of the 3x3 forward with the halo kernel on / off (one pass set per config)
set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6hpmc
for s in "128 28 1" "128 28 0" "256 14 1"; do
  set -- $s
  timeout -s KILL 150 bash tools/diag/run_pmc.sh tools/diag/conv_pmc.py tools/diag/conv_halo_pmc.txt --c $1 --hw $2 --halo $3 --iters 30
  mkdir -p gpurun_out/r6hpmc/c$1_$2_h$3 && mv gpurun_out/pmc_*.csv gpurun_out/pmc.log gpurun_out/r6hpmc/c$1_$2_h$3/
done
