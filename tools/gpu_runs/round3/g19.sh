source tools/gpu_runs/round3/lib.sh
step t_bnbwd 400 $PYT tests/test_conv_bn_bwd_gpu.py tests/test_kernels_gpu.py -k "bnbwd or bn_relu_conv or bottleneck or legacy_lamb"
step m_bnbwd 300 python tools/microbench.py conv-bnbwd
step b_r50 300 python bench.py --json-out gpurun_out/b19_r50.json
step b_r50off 300 env APEX_AMD_CONV_BN_BWD=0 python bench.py --json-out gpurun_out/b19_r50off.json
step d_ddp64 600 env DDP_DIFF_HW=64 python tools/diag/ddp_stats_diff.py
echo done
