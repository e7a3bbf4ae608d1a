#!/usr/bin/env bash
# stock PyTorch-ROCm comparator and the headline path, same box, two runs each
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5stock
rm -rf $out && mkdir -p $out
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --impl stock --steps 20 --warmup 10 --json-out $out/stock_$i.json > $out/stock_$i.log 2>&1
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/amd_$i.json > $out/amd_$i.log 2>&1
done
