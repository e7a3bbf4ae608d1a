#!/usr/bin/env bash
# slab-layout change: its GPU tests, then the same-box A/B and a kernel profile
set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6slab
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_conv_bn_stats_gpu.py tests/test_conv_bn_bwd_gpu.py tests/test_ddp_gpu.py -k "not two_ranks and not bench" > gpurun_out/r6slab/tests.log 2>&1
bash tools/gpu_runs/r6/ab_tree.sh resnet50
bash tools/profile_bench.sh r50_slab 8 --warmup 6
