set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv3x3" > gpurun_out/wg_test.log 2>&1
timeout -k 10 300 python -u tools/microbench.py conv3x3 > gpurun_out/wg_mb.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wg_t -o run -- python3 tools/prof_wgrad.py > gpurun_out/wg_t.log 2>&1
echo ok
