source tools/gpu_runs/round3/lib.sh
T="tests/test_ddp_gpu.py::test_two_ranks_match_concatenated_batch"
step t_ddp_base 300 $PYT "$T"
step t_ddp_noplan 300 env APEX_AMD_STEP_PLAN=0 $PYT "$T"
step t_ddp_nostats 300 env APEX_AMD_CONV_BN_STATS=0 $PYT "$T"
step t_side 300 $PYT tests/test_ddp_gpu.py::test_ddp_side_stream_weight_grads_match_main_stream
echo done
