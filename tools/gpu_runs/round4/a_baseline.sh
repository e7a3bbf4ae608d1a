# round 4, first box: touched GPU tests, headline bench, forced-collective bench with the
# new wire format + SyncBN timing, the standalone conv table
set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_ddp_gpu.py tests/test_conv_bn_bwd_gpu.py tests/test_embedding_gpu.py \
  "tests/test_kernels_gpu.py::test_conv3x3_wgrad_c64_strip_ring" \
  > gpurun_out/r4a/tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 --json-out gpurun_out/r4a/r50.json \
  > gpurun_out/r4a/r50.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 --force-collectives \
  --json-out gpurun_out/r4a/r50fc.json > gpurun_out/r4a/r50fc.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 8 --force-collectives --ddp-bf16-wire fp32 \
  --json-out gpurun_out/r4a/r50fc_fp32.json > gpurun_out/r4a/r50fc_fp32.log 2>&1
timeout -k 10 400 python -u tools/conv_table.py --json gpurun_out/r4a/conv_table.json \
  > gpurun_out/r4a/conv_table.md 2>&1
timeout -k 10 400 python -u tools/conv_variants.py > gpurun_out/r4a/conv_variants.md 2>&1
echo ok
