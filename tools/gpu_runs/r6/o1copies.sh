#!/usr/bin/env bash
# amp O1 weight copies written by FusedAdam: tests + GPT-2-medium A/B (on / off)
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6o1
rm -rf $out && mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convergence_gpu.py -k "gpt2" tests/test_fused_dense_gpu.py > $out/tests.log 2>&1 || timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_convergence_gpu.py -k "gpt2" > $out/tests.log 2>&1
echo tests done
for i in 1 2; do
  for x in 1 0; do
    APEX_AMD_O1_FUSED_COPIES=$x timeout -k 10 300 python -u bench.py --model gpt2_medium --steps 20 --warmup 8 --json-out $out/x${x}_$i.json > $out/x${x}_$i.log 2>&1
  done
done
