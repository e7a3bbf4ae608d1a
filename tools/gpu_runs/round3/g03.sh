source tools/gpu_runs/round3/lib.sh
step t_stats 400 $PYT tests/test_conv_bn_stats_gpu.py
step t_ddp 400 $PYT tests/test_ddp_gpu.py -k "side or forced"
step b_r50 300 python bench.py --json-out gpurun_out/b3_r50.json
step b_r50_nostats 300 env APEX_AMD_CONV_BN_STATS=0 python bench.py --json-out gpurun_out/b3_r50_nostats.json
step b_r50_2 300 python bench.py --json-out gpurun_out/b3_r50_2.json
step b_r50_forced 300 python bench.py --force-collectives --json-out gpurun_out/b3_r50_forced.json
step p_r50 400 bash tools/profile_bench.sh r50stats 8 --warmup 4
echo done
