set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/as_tests.log 2>&1
for r in 1 2; do
  APEX_AMD_PREP_WEIGHTS=0 timeout -k 10 300 python bench.py > gpurun_out/as_off${r}.json 2>> gpurun_out/as.err
  timeout -k 10 300 python bench.py > gpurun_out/as_on${r}.json 2>> gpurun_out/as.err
done
timeout -k 10 500 bash tools/profile_bench.sh r50p 8 --warmup 6
echo ok
