set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest tests/test_bn_persist_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/bnp_tests.log 2>&1
timeout -k 10 300 python tools/microbench.py bn-persist > gpurun_out/bnp_micro.txt 2>&1
APEX_AMD_BN_PERSIST=0 timeout -k 10 300 python bench.py > gpurun_out/bnp_off.json 2> gpurun_out/bnp_bench.err
timeout -k 10 300 python bench.py > gpurun_out/bnp_on.json 2>> gpurun_out/bnp_bench.err
APEX_AMD_BN_PERSIST=0 timeout -k 10 300 python bench.py > gpurun_out/bnp_off2.json 2>> gpurun_out/bnp_bench.err
timeout -k 10 300 python bench.py > gpurun_out/bnp_on2.json 2>> gpurun_out/bnp_bench.err
echo done
