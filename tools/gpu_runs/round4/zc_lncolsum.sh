# round 4 box ZC: LayerNorm gamma/beta column sum with four loads in flight: LN tests,
# kernel stats of short GPT-2 / BERT runs, GPT-2 steps
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4zc
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_determinism_gpu.py -k "layer_norm or ln or determin" > $O/tests.log 2>&1
cd /tmp
for m in gpt2_medium bert_large; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$m -o run -- \
    python3 /root/repo/bench.py --model $m --steps 5 --warmup 3 > /root/repo/$O/prof_$m.log 2>&1
  f=$(find /tmp/prof_$m -name "*kernel_stats.csv" | head -n 1)
  cp "$f" /root/repo/$O/kernel_stats_$m.csv
done
cd /root/repo
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_$r.json > $O/gpt2_$r.log 2>&1
done
echo ok
