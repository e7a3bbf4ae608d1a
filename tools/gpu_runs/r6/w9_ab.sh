#!/usr/bin/env bash
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6w9
mkdir -p $out
for i in 1 2; do
  APEX_AMD_WGRAD9=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/r50_w9_$i.json > $out/r50_w9_$i.log 2>&1
  APEX_AMD_WGRAD9=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/r50_tap_$i.json > $out/r50_tap_$i.log 2>&1
done
