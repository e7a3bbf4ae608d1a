#!/usr/bin/env bash
# rocprofv3 counters for tools/diag/conv_pmc.py (counter run only: no traces besides kernel)
set -eu
repo="$(cd "$(dirname "$0")/../.." && pwd)"
export TMPDIR=/tmp
cd /tmp
rm -rf /tmp/pmc_out
rocprofv3 -i "$repo/tools/diag/conv_pmc.txt" --kernel-trace --output-format csv -d /tmp/pmc_out -o run \
  -- python3 "$repo/tools/diag/conv_pmc.py" > "$repo/gpurun_out/pmc.log" 2>&1
for d in /tmp/pmc_out/pmc_*; do cp "$d/run_counter_collection.csv" "$repo/gpurun_out/pmc_$(basename "$d").csv"; done
ls /tmp/pmc_out -R | head -30 >> "$repo/gpurun_out/pmc.log"
