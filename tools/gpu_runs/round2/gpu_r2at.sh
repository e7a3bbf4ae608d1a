set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_fused_dense_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/at_tests.log 2>&1 || timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/at_tests.log 2>&1
for r in 1 2; do
  APEX_AMD_REDUCE_ONE=0 timeout -k 10 300 python bench.py > gpurun_out/at_off${r}.json 2>> gpurun_out/at.err
  timeout -k 10 300 python bench.py > gpurun_out/at_on${r}.json 2>> gpurun_out/at.err
done
APEX_AMD_REDUCE_ONE=0 timeout -k 10 300 python bench.py --model bert_large > gpurun_out/at_boff.json 2>> gpurun_out/at.err
timeout -k 10 300 python bench.py --model bert_large > gpurun_out/at_bon.json 2>> gpurun_out/at.err
echo ok
