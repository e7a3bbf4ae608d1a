#!/usr/bin/env bash
# same-box A/B of env knobs on one bench model: bash ab_model.sh MODEL "name=ENV=VAL[,ENV=VAL]" ...
set -eu
cd "$GRAFT_REPO_ROOT"
model=$1; shift
out=gpurun_out/r5ab_$model
rm -rf $out && mkdir -p $out
for i in 1 2; do
  for spec in "default=APEX_AMD_X=1" "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env ${envs//,/ } timeout -k 10 300 python -u bench.py --model $model --steps 20 --warmup 8 \
      --json-out $out/${name}_$i.json > $out/${name}_$i.log 2>&1
  done
done
