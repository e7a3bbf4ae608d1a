#!/usr/bin/env bash
# halo kernel tests, per-shape timing, and a same-box ResNet-50 A/B: halo on vs off
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6halo
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_conv_halo_gpu.py > $out/tests.log 2>&1
timeout -k 10 240 python -u tools/diag/halo_bench.py > $out/halo_bench.md 2>&1
for i in 1 2; do
  APEX_AMD_CONV_HALO=1 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/r50_halo_$i.json > $out/r50_halo_$i.log 2>&1
  APEX_AMD_CONV_HALO=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/r50_tap_$i.json > $out/r50_tap_$i.log 2>&1
done
