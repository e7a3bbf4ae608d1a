#!/usr/bin/env bash
# counters of the 1x1 channel-expanding conv forwards (+ BN statistics) at @7 / @14 / @56
set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6c1
for s in "512 2048 7" "256 1024 14" "64 256 56"; do
  set -- $s
  timeout -s KILL 150 bash tools/diag/run_pmc.sh tools/diag/conv1x1_pmc.py tools/diag/conv_l2_pmc.txt --ci $1 --co $2 --hw $3
  mkdir -p gpurun_out/r6c1/c$1_$2_$3 && mv gpurun_out/pmc_*.csv gpurun_out/pmc.log gpurun_out/r6c1/c$1_$2_$3/
done
