source tools/gpu_runs/round3/lib.sh
step d_count 300 python tools/diag/bnbwd_count.py
step t_side 300 $PYT tests/test_ddp_gpu.py::test_ddp_side_stream_weight_grads_match_main_stream
step d_ddpstats 600 python tools/diag/ddp_stats_diff.py
echo done
