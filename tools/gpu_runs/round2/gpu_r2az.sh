cd /root/repo
export PYTHONPATH=.
timeout -k 10 200 python tools/diag/r50_learn.py > gpurun_out/az_default.txt 2>&1
timeout -k 10 200 python tools/diag/r50_learn.py --gemm-tuning off > gpurun_out/az_notune.txt 2>&1
APEX_AMD_GAP_OFF=1 timeout -k 10 200 python tools/diag/r50_learn.py > gpurun_out/az_nogap.txt 2>&1
timeout -k 10 200 python tools/diag/r50_learn.py --no-fused-bn > gpurun_out/az_nofbn.txt 2>&1
timeout -k 10 200 python tools/diag/r50_learn.py --no-gemm-1x1 > gpurun_out/az_nogemm.txt 2>&1
echo ok
