cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python tools/diag/tuned_gemm_validate.py > gpurun_out/bc_validate.txt 2>&1
timeout -k 10 200 python tools/diag/r50_learn.py > gpurun_out/bc_learn.txt 2>&1
echo ok
