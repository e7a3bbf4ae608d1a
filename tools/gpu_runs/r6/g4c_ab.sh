#!/usr/bin/env bash
# 1x1 convs on gemm4w: tests, per-shape bench, ResNet-50 same-box A/B (table vs off)
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6g4c
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_conv_1x1_gemm4w_gpu.py > $out/tests.log 2>&1
for i in 1 2; do
  APEX_AMD_CONV_1X1_G4W=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/r50_g4w_$i.json > $out/r50_g4w_$i.log 2>&1
  APEX_AMD_CONV_1X1_G4W=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/r50_own_$i.json > $out/r50_own_$i.log 2>&1
done
