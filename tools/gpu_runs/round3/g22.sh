source tools/gpu_runs/round3/lib.sh
step t_bnbwd 400 $PYT tests/test_conv_bn_bwd_gpu.py tests/test_conv_bn_stats_gpu.py
step m_bnbwd 300 python tools/microbench.py conv-bnbwd
step m_c1s 300 python tools/microbench.py conv1x1-stats
step b_r50 300 python bench.py --json-out gpurun_out/b22_r50.json
step b_r50all 300 env APEX_AMD_CONV_BN_BWD_MAXM=100000000 python bench.py --json-out gpurun_out/b22_r50all.json
echo done
