source tools/gpu_runs/round3/lib.sh
step t_opt 600 $PYT tests/test_amp_gpu.py tests/test_graph_gpu.py tests/test_amp_guard_gpu.py tests/test_convergence_gpu.py
step p_lnj 300 bash tools/profile_cmd.sh lnj tools/microbench.py ln-join
step h_opt 300 env HOST_PROFILE_OPT_ONLY=1 python tools/diag/host_profile.py --steps 20
step b_r50 300 python bench.py --json-out gpurun_out/b12_r50.json
step b_gpt2 300 python bench.py --model gpt2_medium --json-out gpurun_out/b12_gpt2.json
echo done
