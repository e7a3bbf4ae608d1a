#!/usr/bin/env bash
# ResNet-50 same-box A/B of knobs: bash ab_r50.sh "name=ENV=VAL[,ENV=VAL]" ... (default first)
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5ab_r50
rm -rf $out && mkdir -p $out
for i in 1 2; do
  for spec in "default=APEX_AMD_X=1" "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env ${envs//,/ } timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 \
      --json-out $out/${name}_$i.json > $out/${name}_$i.log 2>&1
  done
done
