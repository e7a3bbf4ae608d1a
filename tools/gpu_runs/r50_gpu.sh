set -e
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem or conv or bn" > gpurun_out/stem_test.log 2>&1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > gpurun_out/r50_bench.log 2>&1
timeout -k 10 400 bash tools/profile_bench.sh r50 8 --warmup 5
echo ok
