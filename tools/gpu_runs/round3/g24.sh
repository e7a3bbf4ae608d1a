source tools/gpu_runs/round3/lib.sh
step t_bnbwd 400 $PYT tests/test_conv_bn_bwd_gpu.py
step m_bnbwd 300 python tools/microbench.py conv-bnbwd
step m_bnbwd_nox 300 env APEX_AMD_BNBWD_DIAG=1 python tools/microbench.py conv-bnbwd
echo done
