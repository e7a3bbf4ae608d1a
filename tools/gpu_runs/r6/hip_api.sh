#!/usr/bin/env bash
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6host
mkdir -p $out
export TMPDIR=/tmp
rm -rf /tmp/prof_api
( cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d /tmp/prof_api -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 8 --warmup 6 ) > $out/api.log 2>&1
python3 tools/diag/hip_api_long.py /tmp/prof_api --min-us 40 > $out/api_long.md
python3 tools/diag/hip_api_long.py /tmp/prof_api --sync > $out/api_sync.txt
python3 tools/diag/gap_attrib.py /tmp/prof_api --last-ms 70 --min-us 25 > $out/gaps.txt
