# round 4 box C: transformer A/Bs with the round-4 DDP defaults (tapered buckets, rsag
# wire, high-priority side stream) - plain vs forced collectives, DDP side stream on/off
# for GPT-2's fp32 dense weight gradients, main-stream priority, gemm8p FFN path
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_$r.json > $O/gpt2_$r.log 2>&1
  timeout -k 10 300 $B --model gpt2_medium --force-collectives --json-out $O/gpt2_fc_$r.json > $O/gpt2_fc_$r.log 2>&1
  APEX_AMD_WGRAD_STREAM_DDP=0 timeout -k 10 300 $B --model gpt2_medium --force-collectives --json-out $O/gpt2_fc_noside_$r.json > $O/gpt2_fc_noside_$r.log 2>&1
  timeout -k 10 300 $B --model gpt2_medium --main-stream-priority high --json-out $O/gpt2_mprio_$r.json > $O/gpt2_mprio_$r.log 2>&1
done
for r in 1 2; do
  timeout -k 10 300 $B --model bert_large --json-out $O/bert_$r.json > $O/bert_$r.log 2>&1
  timeout -k 10 300 $B --model bert_large --force-collectives --json-out $O/bert_fc_$r.json > $O/bert_fc_$r.log 2>&1
done
APEX_AMD_GEMM8P=1 timeout -k 10 300 $B --model bert_large --json-out $O/bert_g8.json > $O/bert_g8.log 2>&1
echo ok
