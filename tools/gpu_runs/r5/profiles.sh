#!/usr/bin/env bash
# Round-5 evidence: ResNet-50 default and side-stream-off (serialized) kernel profiles,
# and the stream -> hardware-queue map of the forced-collective ResNet-50 / GPT-2 steps.
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5prof
mkdir -p $out
export TMPDIR=/tmp
run() {  # name, env, bench args...
  local name=$1 envs=$2; shift 2
  rm -rf /tmp/prof_$name
  ( cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv \
      -d /tmp/prof_$name -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" "$@" ) > $out/$name.log 2>&1
  python3 tools/rocprof_summary.py /tmp/prof_$name --range timed_steps --steps 8 --top 60 \
      --md $out/$name.md --names-out $out/${name}_names.tsv > /dev/null
  python3 tools/diag/queue_map.py /tmp/prof_$name --range timed_steps --md $out/${name}_queues.md > /dev/null
}
run r50 "APEX_AMD_X=1" --steps 8 --warmup 6
run r50ser "APEX_AMD_WGRAD_STREAM=0" --steps 8 --warmup 6
run r50fc "APEX_AMD_X=1" --steps 8 --warmup 6 --force-collectives
run gpt2fc "APEX_AMD_X=1" --model gpt2_medium --steps 8 --warmup 6 --force-collectives
