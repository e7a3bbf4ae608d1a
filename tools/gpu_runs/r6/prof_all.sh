#!/usr/bin/env bash
# serialized ResNet-50 profile (side stream off) with EVERY dispatch listed, current tree
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6pall
rm -rf $out && mkdir -p $out
export TMPDIR=/tmp
rm -rf /tmp/prof_all
( cd /tmp && APEX_AMD_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv \
    -d /tmp/prof_all -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 6 ) > $out/cd.log 2>&1
python3 tools/rocprof_summary.py /tmp/prof_all --range timed_steps --steps 4 --top 80 --md $out/ser.md \
    --names-out $out/ser_names.tsv --dispatch-filter '.' --dispatch-out $out/dispatch.tsv > /dev/null
