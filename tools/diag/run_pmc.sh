#!/usr/bin/env bash
# rocprofv3 counters (counter run only: no traces besides kernel) for one diag script:
#   run_pmc.sh [script.py counters.txt [script args...]]   (default: conv_pmc.py / conv_pmc.txt)
set -eu
repo="$(cd "$(dirname "$0")/../.." && pwd)"
script="${1:-$repo/tools/diag/conv_pmc.py}"
counters="${2:-$repo/tools/diag/conv_pmc.txt}"
shift $(( $# > 2 ? 2 : $# ))
case "$script" in /*) ;; *) script="$repo/$script" ;; esac
case "$counters" in /*) ;; *) counters="$repo/$counters" ;; esac
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/pmc_out
rocprofv3 -i "$counters" --kernel-trace --output-format csv -d /tmp/pmc_out -o run \
  -- python3 "$script" "$@" > "$repo/gpurun_out/pmc.log" 2>&1
for d in /tmp/pmc_out/pmc_*; do cp "$d/run_counter_collection.csv" "$repo/gpurun_out/pmc_$(basename "$d").csv"; done
ls /tmp/pmc_out -R | head -30 >> "$repo/gpurun_out/pmc.log"
