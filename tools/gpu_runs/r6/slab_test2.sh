#!/usr/bin/env bash
set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6slab
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_conv_bn_stats_gpu.py tests/test_conv_bn_bwd_gpu.py > gpurun_out/r6slab/tests2.log 2>&1
timeout -k 10 120 python -u tools/diag/slab_bench.py > gpurun_out/r6slab/slab_bench.md 2>&1
bash tools/gpu_runs/r6/ab_tree.sh resnet50
