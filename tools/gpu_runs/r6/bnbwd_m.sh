#!/usr/bin/env bash
# BN-backward dgrad epilogue on every layer (no M cap) vs the 65,536-pixel cap: ResNet-50 A/B
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6bm2
rm -rf $out && mkdir -p $out
for i in 1 2; do
  for m in 65536 2147483647; do
    APEX_AMD_BNBWD_MAX_M=$m timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/m${m}_$i.json > $out/m${m}_$i.log 2>&1
  done
done
