#!/usr/bin/env bash
# N-fastest order on the halo 3x3 kernel: tests, per-call bench, ResNet-50 A/B (1 vs 0)
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6hnf
rm -rf $out && mkdir -p $out
T="tests/test_conv_bn_stats_gpu.py tests/test_conv_bn_bwd_gpu.py tests/test_conv_halo_gpu.py"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T > $out/tests.log 2>&1
echo tests done
timeout -k 10 300 python -u tools/diag/halo_bench.py > $out/halo_bench.md 2>&1
for i in 1 2; do
  for m in 1 0; do
    APEX_AMD_CONV_HALO_NFAST=$m timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/h${m}_$i.json > $out/h${m}_$i.log 2>&1
  done
done
