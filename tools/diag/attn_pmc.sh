#!/usr/bin/env bash
# rocprofv3 counter passes over tools/diag/attn_pmc.py, one run per pass (counter
# runs carry --kernel-trace only); CSVs -> gpurun_out/attn_pmc_<pass>.csv
set -eu
repo="$(cd "$(dirname "$0")/../.." && pwd)"
export TMPDIR=/tmp
cd /tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
            "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"; do
  i=$((i + 1))
  rm -rf /tmp/apmc
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d /tmp/apmc -o run \
    -- python3 "$repo/tools/diag/attn_pmc.py" > "$repo/gpurun_out/attn_pmc_$i.log" 2>&1
  find /tmp/apmc -name "*counter_collection.csv" -exec cp {} "$repo/gpurun_out/attn_pmc_$i.csv" \;
done
