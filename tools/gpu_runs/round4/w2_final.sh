# round 4 box W2 (after the BN default change): end-of-round benches on the final tree (ResNet-50 twice and under
# forced collectives, BERT-large and GPT-2-medium plain and under forced collectives)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4w2
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/r50_$r.json > $O/r50_$r.log 2>&1
done
timeout -k 10 300 $B --force-collectives --json-out $O/r50fc.json > $O/r50fc.log 2>&1
timeout -k 10 300 $B --model bert_large --json-out $O/bert.json > $O/bert.log 2>&1
timeout -k 10 300 $B --model bert_large --force-collectives --json-out $O/bertfc.json > $O/bertfc.log 2>&1
timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2.json > $O/gpt2.log 2>&1
timeout -k 10 300 $B --model gpt2_medium --force-collectives --json-out $O/gpt2fc.json > $O/gpt2fc.log 2>&1
echo ok
