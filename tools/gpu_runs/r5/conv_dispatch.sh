#!/usr/bin/env bash
# serialized ResNet-50 profile (side stream off) with every conv dispatch listed (grid,
# duration) for the per-call attribution against profiles/r4/conv_table.md
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r5conv
mkdir -p $out
export TMPDIR=/tmp
rm -rf /tmp/prof_cd
( cd /tmp && APEX_AMD_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv \
    -d /tmp/prof_cd -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 6 ) > $out/cd.log 2>&1
python3 tools/rocprof_summary.py /tmp/prof_cd --range timed_steps --steps 4 --top 80 --md $out/ser.md \
    --names-out $out/ser_names.tsv \
    --dispatch-filter 'conv_tap_k|conv3x3_wgrad|wgrad_reduce|stem_|Cijk|splitk|dgrad' --dispatch-out $out/dispatch.tsv > /dev/null
