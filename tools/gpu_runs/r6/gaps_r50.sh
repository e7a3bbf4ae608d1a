#!/usr/bin/env bash
# GPU idle-gap attribution of the ResNet-50 bench step from a kernel-trace-only run
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6host
mkdir -p $out
export TMPDIR=/tmp
rm -rf /tmp/prof_kt
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_kt -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 8 --warmup 6 ) > $out/kt.log 2>&1
python3 tools/diag/gap_attrib.py /tmp/prof_kt --last-ms 66 --min-us 15 > $out/gaps_kt.txt
head -1 $(ls /tmp/prof_kt/*/*kernel_trace.csv /tmp/prof_kt/*kernel_trace.csv 2>/dev/null | head -1) > $out/kt_header.txt || true
python3 tools/diag/timeline_at.py /tmp/prof_kt stem_pad_k --nth 3 --before-ms 2.0 --after-ms 0.3 > $out/timeline_sgd.txt
