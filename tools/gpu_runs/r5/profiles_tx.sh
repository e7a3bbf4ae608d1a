#!/usr/bin/env bash
# transformer kernel profiles (BERT-large, GPT-2-medium) on the round-5 tree
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5prof_tx
mkdir -p $out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  rm -rf /tmp/prof_$name
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv \
      -d /tmp/prof_$name -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" "$@" ) > $out/$name.log 2>&1
  python3 tools/rocprof_summary.py /tmp/prof_$name --range timed_steps --steps 6 --top 50 \
      --md $out/$name.md --names-out $out/${name}_names.tsv > /dev/null
}
run bert --model bert_large --steps 6 --warmup 5
run gpt2 --model gpt2_medium --steps 6 --warmup 5
