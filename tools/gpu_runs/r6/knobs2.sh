#!/usr/bin/env bash
# late-round A/B: main-stream priority, 1x1 weight-gradient split cap
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6knobs2
rm -rf $out && mkdir -p $out
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/base_$i.json > $out/base_$i.log 2>&1
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --main-stream-priority high --json-out $out/prio_$i.json > $out/prio_$i.log 2>&1
  APEX_AMD_WGRAD1X1_SPLITS=64 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/s64_$i.json > $out/s64_$i.log 2>&1
  APEX_AMD_WGRAD1X1_SPLITS=256 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/s256_$i.json > $out/s256_$i.log 2>&1
done
