# round 4 box J: DDP side-stream weight gradients written straight into the (lazily
# zeroed) bucket views instead of fresh tensor + copy - DDP GPU tests, forced-collective
# benches
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_ddp_gpu.py > $O/tests.log 2>&1
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --model gpt2_medium --force-collectives --json-out $O/gpt2_fc_$r.json > $O/gpt2_fc_$r.log 2>&1
  timeout -k 10 300 $B --force-collectives --json-out $O/r50_fc_$r.json > $O/r50_fc_$r.log 2>&1
done
timeout -k 10 300 $B --model bert_large --force-collectives --json-out $O/bert_fc.json > $O/bert_fc.log 2>&1
echo ok
