#!/usr/bin/env bash
# stem BN statistics from the stem conv epilogue: tests + ResNet-50 A/B against ab_old (HEAD)
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6stem
rm -rf $out && mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem or maxpool or bn_relu or resnet" tests/test_models_gpu.py > $out/tests.log 2>&1
echo tests done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/new_$i.json > $out/new_$i.log 2>&1
  timeout -k 10 300 python -u ab_old/bench.py --steps 30 --warmup 10 --json-out $out/old_$i.json > $out/old_$i.log 2>&1
done
