# round 4 box ZH: BN statistics pass with branch-free clamped loads (after ZF: reduce / backward specialised on the ReLU mode,
# clamped loads): BN + determinism tests, kernel stats, ResNet-50 steps
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4zh
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_conv_bn_bwd_gpu.py tests/test_determinism_gpu.py tests/test_ddp_gpu.py \
  -k "bn or batch or norm or determin or sync" > $O/tests.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_zh -o run -- \
  python3 /root/repo/bench.py --steps 5 --warmup 3 > /root/repo/$O/prof.log 2>&1
cd /root/repo
f=$(find /tmp/prof_zh -name "*kernel_stats.csv" | head -n 1)
cp "$f" $O/kernel_stats.csv
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/r50_$r.json > $O/r50_$r.log 2>&1
done
timeout -k 10 300 $B --force-collectives --json-out $O/r50fc.json > $O/r50fc.log 2>&1
echo ok
