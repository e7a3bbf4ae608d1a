source tools/gpu_runs/round3/lib.sh
step t_ddp 400 $PYT tests/test_ddp_gpu.py
step t_tuned 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gemm_tuning_gpu.py
step b_r50_forced 300 python bench.py --force-collectives --json-out gpurun_out/b_r50_forced2.json
step b_r50_forced_noside 300 env APEX_AMD_WGRAD_STREAM_DDP=0 python bench.py --force-collectives --json-out gpurun_out/b_r50_forced_noside.json
step b_r50_forced_nofp32 300 env APEX_AMD_DDP_FP32=0 python bench.py --force-collectives --json-out gpurun_out/b_r50_forced_nofp32.json
step h_opt 300 env HOST_PROFILE_OPT_ONLY=1 python tools/diag/host_profile.py --steps 200
step h_conv 300 python tools/diag/host_profile.py --model convnet --steps 200
echo done
