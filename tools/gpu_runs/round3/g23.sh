source tools/gpu_runs/round3/lib.sh
step m_bnbwd_nox 300 env APEX_AMD_BNBWD_DIAG=1 python tools/microbench.py conv-bnbwd
step m_bnbwd_nb2 300 python tools/microbench.py conv-bnbwd
step m_bnbwd_nb3 300 env APEX_AMD_BNBWD_NB2=0 python tools/microbench.py conv-bnbwd
step t_bnbwd 400 $PYT tests/test_conv_bn_bwd_gpu.py
echo done
