cd /root/repo
export PYTHONPATH=.
timeout -k 10 200 python tools/diag/r50_learn.py > gpurun_out/ba_tuned.txt 2>&1
timeout -k 10 200 python tools/diag/r50_learn.py --gemm-tuning off > gpurun_out/ba_off.txt 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 10 --loss-trace --gemm-tuning off > gpurun_out/ba_bench_off.json 2> gpurun_out/ba.err
echo ok
