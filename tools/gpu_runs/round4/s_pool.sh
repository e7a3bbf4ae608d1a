# round 4 box S: stem max-pool backward, 2x2 input block per thread (default) vs one
# input per thread (APEX_AMD_POOL_BWD1=1): pool tests, kernel stats, ResNet-50 steps
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "maxpool" > $O/tests.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_def -o run -- \
  python3 /root/repo/bench.py --steps 5 --warmup 3 > /root/repo/$O/prof_def.log 2>&1
APEX_AMD_POOL_BWD1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_b1 -o run -- \
  python3 /root/repo/bench.py --steps 5 --warmup 3 > /root/repo/$O/prof_b1.log 2>&1
cd /root/repo
for v in def b1; do
  f=$(find /tmp/prof_$v -name "*kernel_stats.csv" | head -n 1)
  grep -i "maxpool" "$f" > $O/pool_stats_$v.csv || true
done
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/r50_def_$r.json > $O/r50_def_$r.log 2>&1
  APEX_AMD_POOL_BWD1=1 timeout -k 10 300 $B --json-out $O/r50_b1_$r.json > $O/r50_b1_$r.log 2>&1
done
echo ok
