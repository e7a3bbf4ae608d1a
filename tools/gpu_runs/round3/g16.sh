source tools/gpu_runs/round3/lib.sh
step t_bnbwd 400 $PYT tests/test_conv_bn_bwd_gpu.py
step t_conv 400 $PYT tests/test_conv_bn_stats_gpu.py tests/test_ddp_gpu.py::test_ddp_side_stream_weight_grads_match_main_stream
step b_r50 300 python bench.py --json-out gpurun_out/b16_r50.json
step b_r50off 300 env APEX_AMD_CONV_BN_BWD=0 python bench.py --json-out gpurun_out/b16_r50off.json
step d_ddpstats 600 python tools/diag/ddp_stats_diff.py
echo done
