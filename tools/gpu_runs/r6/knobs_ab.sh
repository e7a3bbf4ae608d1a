#!/usr/bin/env bash
# re-check two off-by-default A/B switches on the late-round tree: gemm4w 1x1 routing and the
# strip-ring 3x3 weight gradient on channel tiles
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6knobs
rm -rf $out && mkdir -p $out
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/base_$i.json > $out/base_$i.log 2>&1
  APEX_AMD_CONV_1X1_G4W=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/g4w_$i.json > $out/g4w_$i.log 2>&1
  APEX_AMD_WGRAD9=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/w9_$i.json > $out/w9_$i.log 2>&1
done
