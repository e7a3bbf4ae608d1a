# round 4 box H: end-of-round evidence on the final tree - ResNet-50 bench (two runs +
# forced collectives), BERT / GPT-2 benches, rocprofv3 kernel tables
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/r50_$r.json > $O/r50_$r.log 2>&1
done
timeout -k 10 300 $B --force-collectives --json-out $O/r50fc.json > $O/r50fc.log 2>&1
timeout -k 10 300 $B --model bert_large --json-out $O/bert.json > $O/bert.log 2>&1
timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2.json > $O/gpt2.log 2>&1
timeout -k 10 240 bash tools/profile_bench.sh r50 10 --warmup 5
timeout -k 10 240 bash tools/profile_bench.sh r50fc 10 --warmup 5 --force-collectives
echo ok
