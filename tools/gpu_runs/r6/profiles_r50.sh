#!/usr/bin/env bash
# Round-6 ResNet-50 kernel profiles: default (side stream on) and serialized (side stream
# off) with every conv dispatch listed
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6prof
mkdir -p $out
timeout -k 10 400 bash tools/profile_bench.sh resnet50_r6 10 --warmup 6
mv gpurun_out/prof_resnet50_r6.md gpurun_out/prof_resnet50_r6_names.tsv gpurun_out/prof_resnet50_r6.log $out/
export TMPDIR=/tmp
rm -rf /tmp/prof_cd
( cd /tmp && APEX_AMD_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv \
    -d /tmp/prof_cd -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 6 ) > $out/cd.log 2>&1
python3 tools/rocprof_summary.py /tmp/prof_cd --range timed_steps --steps 4 --top 80 --md $out/ser.md \
    --names-out $out/ser_names.tsv \
    --dispatch-filter 'conv_tap_k|conv3h_k|conv3x3_wgrad|wgrad_reduce|stem_|Cijk|splitk|dgrad|gemm4w|wgrad4w' --dispatch-out $out/dispatch.tsv > /dev/null
