#!/usr/bin/env bash
# serialized ResNet-50 profiles with the X2 BN backward fusion on / off (per-kernel times)
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6x2p
rm -rf $out && mkdir -p $out
export TMPDIR=/tmp
for x in 1 0; do
  rm -rf /tmp/prof_x2
  ( cd /tmp && APEX_AMD_BN_X2=$x APEX_AMD_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv \
      -d /tmp/prof_x2 -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 4 --warmup 6 ) > $out/cd_$x.log 2>&1
  python3 tools/rocprof_summary.py /tmp/prof_x2 --range timed_steps --steps 4 --top 80 --md $out/ser_$x.md \
      --names-out $out/ser_names_$x.tsv --dispatch-filter '.' --dispatch-out $out/dispatch_$x.tsv > /dev/null
done
