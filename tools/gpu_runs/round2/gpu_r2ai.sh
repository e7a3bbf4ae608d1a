set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ai.log 2>&1
for m in bert_large gpt2_medium resnet50; do
  timeout -k 10 200 python tools/diag/plan_cache.py --model $m > gpurun_out/plan2_$m.txt 2>&1
  timeout -k 10 300 python bench.py --model $m > gpurun_out/ai_$m.json 2>> gpurun_out/ai.err
  timeout -k 10 300 python bench.py --model $m > gpurun_out/ai2_$m.json 2>> gpurun_out/ai.err
done
timeout -k 10 500 bash tools/profile_bench.sh bert3 4 --model bert_large --warmup 4
echo ok
