set -e
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py -k "bias_grad or bert or gpt2" > gpurun_out/tx_test.log 2>&1
timeout -k 10 400 python -u bench.py --model gpt2_medium --steps 10 --warmup 5 > gpurun_out/gpt2_bench.log 2>&1
timeout -k 10 400 bash tools/profile_bench.sh gpt2 4 --model gpt2_medium --warmup 3
echo ok
