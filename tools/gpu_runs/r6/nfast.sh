#!/usr/bin/env bash
# N-fastest conv tile order: conv tests (default mode 1, then mode 2), per-call bench,
# ResNet-50 same-box A/B (modes 1 / 0 / 2)
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6nf
rm -rf $out && mkdir -p $out
T="tests/test_conv_bn_stats_gpu.py tests/test_conv_bn_bwd_gpu.py tests/test_conv_halo_gpu.py tests/test_conv_1x1_gemm4w_gpu.py"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > $out/tests1.log 2>&1
echo tests1 done
APEX_AMD_CONV_NFAST=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > $out/tests2.log 2>&1
echo tests2 done
timeout -k 10 200 python -u tools/diag/nfast_bench.py > $out/bench.md 2>&1
for i in 1 2; do
  for m in 1 0 2; do
    APEX_AMD_CONV_NFAST=$m timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/m${m}_$i.json > $out/m${m}_$i.log 2>&1
  done
done
