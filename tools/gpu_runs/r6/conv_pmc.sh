#!/usr/bin/env bash
# L2 traffic / MFMA busy of the 3x3 forward conv at the ResNet-50 shapes (one pass set each)
set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6pmc
for s in "128 28" "64 56" "256 14"; do
  set -- $s
  timeout -s KILL 150 bash tools/diag/run_pmc.sh tools/diag/conv_pmc.py tools/diag/conv_l2_pmc.txt --c $1 --hw $2 --iters 30
  mkdir -p gpurun_out/r6pmc/c$1_$2 && mv gpurun_out/pmc_*.csv gpurun_out/pmc.log gpurun_out/r6pmc/c$1_$2/
done
