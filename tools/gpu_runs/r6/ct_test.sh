#!/usr/bin/env bash
# C^T epilogue: conv tests, per-shape benches, ResNet-50 A/B against ab_old (previous build)
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6ct
mkdir -p $out
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_conv_bn_stats_gpu.py tests/test_conv_bn_bwd_gpu.py tests/test_conv_halo_gpu.py \
  tests/test_conv_1x1_gemm4w_gpu.py > $out/tests.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_kernels_gpu.py -k "conv" > $out/tests_kernels.log 2>&1
timeout -k 10 200 python -u tools/diag/halo_bench.py > $out/halo_bench.md 2>&1
timeout -k 10 200 python -u tools/diag/bnbwd1x1_bench.py 1 > $out/bnbwd.md 2>&1
bash tools/gpu_runs/r6/ab_tree.sh resnet50
