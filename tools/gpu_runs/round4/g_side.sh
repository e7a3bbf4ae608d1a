# round 4 box G: side-stream priority / lag for the transformer dense weight gradients
# (plain single-GPU runs), two runs each
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_def_$r.json > $O/gpt2_def_$r.log 2>&1
  APEX_AMD_WGRAD_STREAM_PRIO=high timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_hi_$r.json > $O/gpt2_hi_$r.log 2>&1
  APEX_AMD_WGRAD_STREAM_PRIO=high APEX_AMD_WGRAD_LAG=4 timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_hilag_$r.json > $O/gpt2_hilag_$r.log 2>&1
  timeout -k 10 300 $B --model bert_large --json-out $O/bert_def_$r.json > $O/bert_def_$r.log 2>&1
  APEX_AMD_DENSE_SIDE=all APEX_AMD_WGRAD_STREAM_PRIO=high timeout -k 10 300 $B --model bert_large --json-out $O/bert_allhi_$r.json > $O/bert_allhi_$r.log 2>&1
done
echo ok
