#!/usr/bin/env bash
# same-box A/B of the halo conv's pixel-tile choice: cost model (224 or 256) vs 256 only
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6bm
rm -rf $out && mkdir -p $out
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/auto_$i.json > $out/auto_$i.log 2>&1
  APEX_AMD_CONV_HALO_BM=256 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/bm256_$i.json > $out/bm256_$i.log 2>&1
done
