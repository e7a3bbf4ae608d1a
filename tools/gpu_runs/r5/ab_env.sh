#!/usr/bin/env bash
# same-box A/B of an environment knob: bash ab_env.sh MODEL VAR ON OFF (two runs per side,
# interleaved) -> gpurun_out/r5abenv_MODEL/{on,off}_{1,2}.json
set -eu
cd "$GRAFT_REPO_ROOT"
model=$1; var=$2; on=$3; off=$4
out=gpurun_out/r5abenv_$model
rm -rf $out && mkdir -p $out
for i in 1 2; do
  for v in on off; do
    val=$on; [ $v = off ] && val=$off
    env $var=$val timeout -k 10 300 python -u bench.py --model $model --steps 20 --warmup 8 \
      --json-out $out/${v}_$i.json > $out/${v}_$i.log 2>&1
  done
done
