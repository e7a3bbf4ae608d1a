#!/usr/bin/env bash
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6host
mkdir -p $out
export TMPDIR=/tmp
rm -rf /tmp/prof_hl
( cd /tmp && APEX_AMD_BENCH_STEP_MARKS=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv \
    -d /tmp/prof_hl -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 6 ) > $out/hl.log 2>&1
ls -R /tmp/prof_hl | head -20 > $out/hl_files.txt
head -3 /tmp/prof_hl/run_marker_api_trace.csv > $out/marker_header.txt || true
python3 tools/diag/host_lead.py /tmp/prof_hl > $out/host_lead.md
