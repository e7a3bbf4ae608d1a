# round 4 box O: attention tile DMA with scalar tile bases + 32-bit lane offsets
# (default) vs per-lane 64-bit addresses (APEX_AMD_ATTN_ADDR64=1): kernel tests, the
# native-call microbench and BERT-large / GPT-2-medium steps, two runs each
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_attention_gpu.py > $O/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 300 python -u tools/microbench.py attn --quick > $O/mb_$r.txt 2>&1
done
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --model bert_large --json-out $O/bert_def_$r.json > $O/bert_def_$r.log 2>&1
  APEX_AMD_ATTN_ADDR64=1 timeout -k 10 300 $B --model bert_large --json-out $O/bert_a64_$r.json > $O/bert_a64_$r.log 2>&1
  timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_def_$r.json > $O/gpt2_def_$r.log 2>&1
  APEX_AMD_ATTN_ADDR64=1 timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_a64_$r.json > $O/gpt2_a64_$r.log 2>&1
done
echo ok
