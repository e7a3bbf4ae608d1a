#!/usr/bin/env bash
# Round-6 transformer kernel profiles (default streams) + plain bench numbers
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6prof
mkdir -p $out
for m in gpt2_medium bert_large; do
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 8 --json-out $out/$m.json > $out/$m.log 2>&1
  timeout -k 10 400 bash tools/profile_bench.sh ${m}_r6 8 --model $m --warmup 6
  mv gpurun_out/prof_${m}_r6.md gpurun_out/prof_${m}_r6_names.tsv gpurun_out/prof_${m}_r6.log $out/
done
