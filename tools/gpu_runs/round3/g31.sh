source tools/gpu_runs/round3/lib.sh
step t_attn2 300 env APEX_AMD_ATTN_FWD=2 $PYT tests/test_attention_gpu.py
step mb_attn 300 python tools/microbench.py attn --quick
step t_ddp 600 $PYT tests/test_ddp_gpu.py
step b_fc 400 python bench.py --force-collectives --json-out gpurun_out/b31_fc.json
step b_fcs 400 env APEX_AMD_WGRAD_STREAM_DDP=1 python bench.py --force-collectives --json-out gpurun_out/b31_fcs.json
step p_fc 500 bash tools/profile_bench.sh r50fc3 6 --warmup 4 --force-collectives
echo done
