set -e
cd /root/repo
mkdir -p gpurun_out
rc=0
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_q.log 2>&1 || rc=$?
if [ $rc -ne 0 ]; then echo "attention tests rc=$rc: stopping"; exit $rc; fi
APEX_AMD_ATTN_BASE=1 PYTHONPATH=. timeout -k 10 300 python -u tools/microbench.py attn > gpurun_out/mb_attn_base.txt 2>&1
PYTHONPATH=. timeout -k 10 300 python -u tools/microbench.py attn > gpurun_out/mb_attn.txt 2>&1
timeout -k 10 300 python bench.py --model bert_large --steps 10 --warmup 5 > gpurun_out/bench_bert.json 2> gpurun_out/bench_bert.log
APEX_AMD_ATTN_BASE=1 timeout -k 10 300 python bench.py --model bert_large --steps 10 --warmup 5 > gpurun_out/bench_bert_base.json 2>> gpurun_out/bench_bert.log
timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 5 > gpurun_out/bench_gpt2.json 2> gpurun_out/bench_gpt2.log
APEX_AMD_ATTN_BASE=1 timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 5 > gpurun_out/bench_gpt2_base.json 2>> gpurun_out/bench_gpt2.log
echo "done"
