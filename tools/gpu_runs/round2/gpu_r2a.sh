set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 180 --timeout-method thread > gpurun_out/ddp_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 15 --loss-trace > gpurun_out/r50_amd_trace.json 2> gpurun_out/r50_amd_trace.log
timeout -k 10 300 python bench.py --steps 10 --warmup 15 --loss-trace --impl stock > gpurun_out/r50_stock_trace.json 2> gpurun_out/r50_stock_trace.log
echo done
