#!/usr/bin/env bash
# X2 fusion with the channel-major slab: tests (forced on), serialized profiles on / off,
# ResNet-50 A/B on / off
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6x2b
rm -rf $out && mkdir -p $out
APEX_AMD_BN_X2=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_bn_x2_gpu.py tests/test_models_gpu.py -k "x2 or resnet" > $out/tests.log 2>&1
echo tests done
bash tools/gpu_runs/r6/x2_prof.sh
mv gpurun_out/r6x2p/ser_*.md $out/
for i in 1 2; do
  for x in 1 0; do
    APEX_AMD_BN_X2=$x timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/x${x}_$i.json > $out/x${x}_$i.log 2>&1
  done
done
