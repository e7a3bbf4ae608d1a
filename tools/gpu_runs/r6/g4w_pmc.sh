#!/usr/bin/env bash
# gemm4w tests after the variant cleanup + L2 counters of the 3x3 conv shapes
set -eu
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r6g
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm4w_gpu.py > gpurun_out/r6g/tests.log 2>&1
bash tools/gpu_runs/r6/conv_pmc.sh
