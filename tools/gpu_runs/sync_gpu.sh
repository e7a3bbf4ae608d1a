set -e
cd /root/repo
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ddp_gpu.py > gpurun_out/sync_test.log 2>&1
echo ok
