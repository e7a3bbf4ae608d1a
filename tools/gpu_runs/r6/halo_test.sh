#!/usr/bin/env bash
set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6halo
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_conv_halo_gpu.py > gpurun_out/r6halo/tests.log 2>&1
timeout -k 10 240 python -u tools/diag/halo_bench.py > gpurun_out/r6halo/halo_bench.md 2>&1
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
  tests/test_conv_bn_stats_gpu.py tests/test_conv_bn_bwd_gpu.py > gpurun_out/r6halo/tests_conv.log 2>&1
