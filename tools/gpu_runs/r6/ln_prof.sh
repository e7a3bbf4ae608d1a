#!/usr/bin/env bash
# per-kernel times of the LayerNorm join backward: per-wave LDS rows (default) vs one row set
set -eu
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r6lnp
rm -rf $out && mkdir -p $out
for one in 0 1; do
  ( cd /tmp && LN_ONE_ROW=$one timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d /tmp/lnp_$one -o run -- python3 "$GRAFT_REPO_ROOT/tools/diag/ln_bwd_bench.py" ) > $out/bench_$one.md 2>&1
  find /tmp/lnp_$one -name "*kernel_stats.csv" -exec cp {} $out/stats_$one.csv \;
done
