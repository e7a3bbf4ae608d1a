#!/usr/bin/env bash
# Kernel-trace any Python tool under rocprofv3 on the GPU box and summarise every
# kernel it ran into gpurun_out/prof_<name>.md (raw traces stay in /tmp).
#   tools/profile_cmd.sh <name> <script.py> [args...]
set -eu
name="$1"; shift
repo="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$repo/gpurun_out"
export TMPDIR=/tmp
script="$1"; shift
case "$script" in /*) ;; *) script="$repo/$script" ;; esac
cd /tmp
rm -rf "/tmp/prof_$name"
rocprofv3 --kernel-trace --output-format csv -d "/tmp/prof_$name" -o run \
  -- python3 "$script" "$@" > "$repo/gpurun_out/prof_$name.log" 2>&1
python3 "$repo/tools/rocprof_summary.py" "/tmp/prof_$name" --steps 1 --top 30 \
  --md "$repo/gpurun_out/prof_$name.md"
