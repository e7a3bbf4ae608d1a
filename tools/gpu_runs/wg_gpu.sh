set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > gpurun_out/wg_test.log 2>&1
timeout -k 10 300 python -u tools/microbench.py conv-s2 > gpurun_out/s2_mb.log 2>&1
timeout -k 10 300 python -u tools/microbench.py conv3x3 > gpurun_out/wg_mb.log 2>&1
echo ok
