cd /root/repo
export PYTHONPATH=.
timeout -k 10 200 python tools/diag/tuned_gemm_check.py > gpurun_out/bb_tuned.txt 2>&1
timeout -k 10 200 python tools/diag/tuned_gemm_check.py --gemm-tuning off > gpurun_out/bb_off.txt 2>&1
echo ok
