set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/diag/ddp_parity.py > gpurun_out/ddp_parity.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --warmup 15 --loss-trace > gpurun_out/r50_amd_trace.json 2> gpurun_out/r50_amd_trace.log
timeout -k 10 300 python bench.py --steps 10 --warmup 15 --loss-trace --impl stock > gpurun_out/r50_stock_trace.json 2> gpurun_out/r50_stock_trace.log
timeout -k 10 300 python bench.py --steps 10 --warmup 15 --loss-trace --lr 0.02 > gpurun_out/r50_amd_trace2.json 2>> gpurun_out/r50_amd_trace.log
timeout -k 10 300 python bench.py --steps 10 --warmup 15 --loss-trace --impl stock --lr 0.02 > gpurun_out/r50_stock_trace2.json 2>> gpurun_out/r50_stock_trace.log
echo done
