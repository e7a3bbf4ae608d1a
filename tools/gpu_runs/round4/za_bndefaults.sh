# round 4 box ZA: new BN grid defaults (red_rpt 32, elem_rpt 8) vs the old ones
# (APEX_AMD_BN_TUNING="64,-1,-1,16,-1,-1"): BN tests, ResNet-50 two runs each
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4za
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_conv_bn_bwd_gpu.py tests/test_determinism_gpu.py \
  -k "bn or batch or norm or determin" > $O/tests.log 2>&1
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/new_$r.json > $O/new_$r.log 2>&1
  APEX_AMD_BN_TUNING="64,-1,-1,16,-1,-1" timeout -k 10 300 $B --json-out $O/old_$r.json > $O/old_$r.log 2>&1
done
echo ok
