set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "attn or attention or gpt2 or bert" > gpurun_out/gputests_u.log 2>&1
timeout -k 10 300 python tools/microbench.py attn > gpurun_out/mb_attn_u.txt 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_r50_u.json 2> gpurun_out/bench_r50_u.log
timeout -k 10 300 python bench.py --model bert_large > gpurun_out/bench_bert_u.json 2> gpurun_out/bench_bert_u.log
timeout -k 10 300 python bench.py --model gpt2_medium > gpurun_out/bench_gpt2_u.json 2> gpurun_out/bench_gpt2_u.log
echo done
