source tools/gpu_runs/round3/lib.sh
step t_stats 400 $PYT tests/test_conv_bn_stats_gpu.py
step mb_stats 300 python tools/microbench.py conv1x1-stats
step b_stats 300 python bench.py --json-out gpurun_out/b6_stats.json
step b_nostats 300 env APEX_AMD_CONV_BN_STATS=0 python bench.py --json-out gpurun_out/b6_nostats.json
step b_stats2 300 python bench.py --json-out gpurun_out/b6_stats2.json
step p_r50 400 bash tools/profile_bench.sh r50stats2 8 --warmup 4
echo done
