# round 4 box U/V: BN apply / backward (U) and reduce (V) passes with the per-channel constants staged in
# LDS per workgroup: BN tests, kernel stats of a short ResNet-50 run, ResNet-50 steps
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_conv_bn_bwd_gpu.py -k "bn or batch or norm or maxpool" > $O/tests.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_v -o run -- \
  python3 /root/repo/bench.py --steps 5 --warmup 3 > /root/repo/$O/prof.log 2>&1
cd /root/repo
f=$(find /tmp/prof_v -name "*kernel_stats.csv" | head -n 1)
cp "$f" $O/kernel_stats.csv
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/r50_$r.json > $O/r50_$r.log 2>&1
done
echo ok
