set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_amp_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/bf_tests.log 2>&1
for m in bert_large gpt2_medium; do
  for r in 1 2; do
    APEX_AMD_WGRAD_STREAM=0 timeout -k 10 300 python bench.py --model $m --loss-trace > gpurun_out/bf_off${r}_$m.json 2>> gpurun_out/bf.err
    timeout -k 10 300 python bench.py --model $m --loss-trace > gpurun_out/bf_on${r}_$m.json 2>> gpurun_out/bf.err
  done
done
echo ok
