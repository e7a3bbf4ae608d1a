set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest tests/test_bn_persist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bnp_tests2.log 2>&1
timeout -k 10 300 python tools/microbench.py bn-persist --quick > gpurun_out/bnp_micro2.txt 2>&1
echo done
