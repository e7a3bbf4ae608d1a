set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_amp_gpu.py tests/test_models_gpu.py tests/test_optimizers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_aj.log 2>&1 || timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_amp_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_aj.log 2>&1
for m in bert_large gpt2_medium resnet50; do
  timeout -k 10 200 python tools/diag/plan_cache.py --model $m > gpurun_out/plan3_$m.txt 2>&1
  timeout -k 10 300 python bench.py --model $m > gpurun_out/aj_$m.json 2>> gpurun_out/aj.err
done
timeout -k 10 500 bash tools/profile_bench.sh bert4 4 --model bert_large --warmup 4
echo ok
