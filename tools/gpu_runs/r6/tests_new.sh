#!/usr/bin/env bash
# new round-6 GPU tests (side-stream wait hooks, N>1 self-check) + the headline bench
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6t
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread \
  tests/test_side_stream_gpu.py tests/test_ddp_gpu.py -k "bench or side_stream or penalty" > $out/tests.log 2>&1
timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --json-out $out/amd_r50.json > $out/amd_r50.log 2>&1
