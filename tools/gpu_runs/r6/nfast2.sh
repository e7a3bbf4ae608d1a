#!/usr/bin/env bash
# N-fastest tile order by shape (mode 1) vs everywhere (2) vs off (0): tests + ResNet-50 A/B
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6nf3
rm -rf $out && mkdir -p $out
T="tests/test_conv_bn_stats_gpu.py tests/test_conv_bn_bwd_gpu.py tests/test_conv_halo_gpu.py tests/test_kernels_gpu.py"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T -k "conv or bn" > $out/tests.log 2>&1
echo tests done
for i in 1 2; do
  for m in 1 0 2; do
    APEX_AMD_CONV_NFAST=$m timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/m${m}_$i.json > $out/m${m}_$i.log 2>&1
  done
done
