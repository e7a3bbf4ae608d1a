#!/usr/bin/env bash
# stride-2 3x3 dgrad with the BN-backward epilogue: tests + ResNet-50 A/B vs ab_old
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6s2
rm -rf $out && mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_conv_bn_bwd_gpu.py tests/test_models_gpu.py tests/test_bn_x2_gpu.py > $out/tests.log 2>&1
echo tests done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/new_$i.json > $out/new_$i.log 2>&1
  timeout -k 10 300 python -u ab_old/bench.py --steps 30 --warmup 10 --json-out $out/old_$i.json > $out/old_$i.log 2>&1
done
