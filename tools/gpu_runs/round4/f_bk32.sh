# round 4 box F: 32-deep K-tile conv ring (auto from 1024 workgroups) - microbench,
# conv GPU tests, ResNet-50 A/B against the 64-deep ring
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 300 python tools/conv_variants.py --variants default bk32off bk32w64 > $O/variants.md 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_conv_bn_bwd_gpu.py tests/test_conv_bn_stats_gpu.py \
  tests/test_models_gpu.py > $O/tests.log 2>&1
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/r50_auto_$r.json > $O/r50_auto_$r.log 2>&1
  APEX_AMD_CONV_BK32=0 timeout -k 10 300 $B --json-out $O/r50_off_$r.json > $O/r50_off_$r.log 2>&1
  APEX_AMD_CONV_BK32_64=1 timeout -k 10 300 $B --json-out $O/r50_w64_$r.json > $O/r50_w64_$r.log 2>&1
done
echo ok
