#!/usr/bin/env bash
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6tap1
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_conv_bn_bwd_gpu.py tests/test_conv_bn_stats_gpu.py > $out/tests.log 2>&1
timeout -k 10 200 python -u tools/diag/conv1x1_g4w_bench.py > $out/new_1x1.md 2>&1
( cd ab_old && timeout -k 10 200 python -u ../tools/diag/conv1x1_g4w_bench.py > ../$out/old_1x1.md 2>&1 ) || true
bash tools/gpu_runs/r6/ab_tree.sh resnet50
