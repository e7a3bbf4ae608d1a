set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "maxpool or pool or bn_relu_maxpool or mt_plan" > gpurun_out/pool_tests.log 2>&1
for r in 1 2; do
  APEX_AMD_POOL_GENERIC=1 timeout -k 10 300 python bench.py > gpurun_out/an_gen${r}.json 2>> gpurun_out/an.err
  timeout -k 10 300 python bench.py > gpurun_out/an_new${r}.json 2>> gpurun_out/an.err
done
timeout -k 10 500 bash tools/profile_bench.sh r50 8 --warmup 6
echo ok
