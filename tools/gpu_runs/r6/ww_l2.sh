#!/usr/bin/env bash
# L2 counters of wgrad4w at the GPT-2 / BERT FFN shapes
set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6ww
for s in "8192 4096 1024 2" "8192 1024 4096 2" "16384 4096 1024 4"; do
  set -- $s
  timeout -s KILL 150 bash tools/diag/run_pmc.sh tools/diag/ww_pmc.py tools/diag/conv_l2_pmc.txt --t $1 --m $2 --n $3 --splits $4
  mkdir -p gpurun_out/r6ww/t$1_m$2_n$3_s$4 && mv gpurun_out/pmc_*.csv gpurun_out/pmc.log gpurun_out/r6ww/t$1_m$2_n$3_s$4/
done
