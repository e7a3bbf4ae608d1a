source tools/gpu_runs/round3/lib.sh
step d_count 300 python tools/diag/bnbwd_count.py
step t_bnbwd 400 $PYT tests/test_conv_bn_bwd_gpu.py -k bottleneck
step p_on 400 bash tools/profile_bench.sh r50bnbwd 8 --warmup 4
step p_off 400 env APEX_AMD_CONV_BN_BWD=0 bash tools/profile_bench.sh r50bnbwdoff 8 --warmup 4
step d_ddpstats 600 python tools/diag/ddp_stats_diff.py
echo done
