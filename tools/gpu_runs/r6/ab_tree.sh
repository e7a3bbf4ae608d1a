#!/usr/bin/env bash
# same-box A/B of this tree ("new") against a snapshot of the previous commit built into
# ab_old/ ("old": its own package, .so, bench.py and GEMM tables), two runs each
set -eu
cd "$GRAFT_REPO_ROOT"
model=${1:-resnet50}
out=gpurun_out/r6ab_$model
rm -rf $out && mkdir -p $out
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model $model --steps 30 --warmup 10 --json-out $out/new_$i.json > $out/new_$i.log 2>&1
  timeout -k 10 300 python -u ab_old/bench.py --model $model --steps 30 --warmup 10 --json-out $out/old_$i.json > $out/old_$i.log 2>&1
done
