#!/usr/bin/env bash
# same-box A/B of two builds of the extension: bash ab_so.sh MODEL (ab_so/{new,old}.so,
# swapped into this scratch copy of the tree before each run)
set -eu
cd "$GRAFT_REPO_ROOT"
model=$1
so=apex_example_amd/_C.cpython-310-x86_64-linux-gnu.so
out=gpurun_out/r5abso_$model
rm -rf $out && mkdir -p $out
for i in 1 2; do
  for v in new old; do
    cp ab_so/$v.so $so
    timeout -k 10 300 python -u bench.py --model $model --steps 20 --warmup 8 \
      --json-out $out/${v}_$i.json > $out/${v}_$i.log 2>&1
  done
done
cp ab_so/new.so $so
