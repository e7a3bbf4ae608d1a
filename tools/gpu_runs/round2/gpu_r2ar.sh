set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ar_tests.log 2>&1
for r in 1 2; do
  git_rev=x
  timeout -k 10 300 python bench.py > gpurun_out/ar_new${r}.json 2>> gpurun_out/ar.err
done
timeout -k 10 500 bash tools/profile_bench.sh r50t 8 --warmup 6
echo ok
