# round 4 box K: GPT-2 / BERT knob re-checks on the final tree (LayerNorm backward grid
# cap, split-K dense wgrads, software-pipelined attention forward), two runs each
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_def_$r.json > $O/gpt2_def_$r.log 2>&1
  APEX_AMD_LN_BWD_BLOCKS=2048 timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_ln2048_$r.json > $O/gpt2_ln2048_$r.log 2>&1
  APEX_AMD_LN_BWD_BLOCKS=512 timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_ln512_$r.json > $O/gpt2_ln512_$r.log 2>&1
  APEX_AMD_DENSE_SPLITK=0 timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_nosplit_$r.json > $O/gpt2_nosplit_$r.log 2>&1
  timeout -k 10 300 $B --model bert_large --json-out $O/bert_def_$r.json > $O/bert_def_$r.log 2>&1
  APEX_AMD_ATTN_FWD=2 timeout -k 10 300 $B --model bert_large --json-out $O/bert_fwd2_$r.json > $O/bert_fwd2_$r.log 2>&1
done
echo ok
