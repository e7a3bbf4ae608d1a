#!/usr/bin/env bash
# Profile bench.py under rocprofv3 (kernel trace + roctx markers) on the GPU box
# and summarise the timed steps into gpurun_out/prof_<name>.md.  Raw traces stay
# in /tmp (they exceed gpurun's merge limit).
#   tools/profile_bench.sh <name> <steps> [bench.py args...]
set -eu
name="$1"; steps="$2"; shift 2
repo="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$repo/gpurun_out"
export TMPDIR=/tmp
cd /tmp
rm -rf "/tmp/prof_$name"
rocprofv3 --kernel-trace --marker-trace --output-format csv -d "/tmp/prof_$name" -o run \
  -- python3 "$repo/bench.py" --steps "$steps" "$@" > "$repo/gpurun_out/prof_$name.log" 2>&1
python3 "$repo/tools/rocprof_summary.py" "/tmp/prof_$name" --range timed_steps --steps "$steps" \
  --top 45 --gaps 25 --md "$repo/gpurun_out/prof_$name.md" --names-out "$repo/gpurun_out/prof_${name}_names.tsv"
