#!/usr/bin/env bash
# full GPU suite (no -x: every failure listed) + the headline bench
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6suite
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 150 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/tests.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --json-out $out/r50.json > $out/r50.log 2>&1
fi
exit $rc
