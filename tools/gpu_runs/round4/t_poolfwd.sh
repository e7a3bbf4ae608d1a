# round 4 box T: stem BN+ReLU+max-pool forward with the BN scale/shift staged in LDS:
# pool tests, kernel stats of a short ResNet-50 run, ResNet-50 steps
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "maxpool" > $O/tests.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_t -o run -- \
  python3 /root/repo/bench.py --steps 5 --warmup 3 > /root/repo/$O/prof.log 2>&1
cd /root/repo
f=$(find /tmp/prof_t -name "*kernel_stats.csv" | head -n 1)
cp "$f" $O/kernel_stats.csv
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/r50_$r.json > $O/r50_$r.log 2>&1
done
echo ok
