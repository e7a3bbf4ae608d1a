source tools/gpu_runs/round3/lib.sh
step t_stats 400 $PYT tests/test_conv_bn_stats_gpu.py
step t_guard 400 $PYT tests/test_amp_guard_gpu.py
step mb_stats 300 python tools/microbench.py conv1x1-stats
step b_stats 300 python bench.py --json-out gpurun_out/b7_stats.json
step b_nostats 300 env APEX_AMD_CONV_BN_STATS=0 python bench.py --json-out gpurun_out/b7_nostats.json
step b_conv_sgd 200 python bench.py --model convnet --steps 200 --warmup 30 --json-out gpurun_out/b7_conv_sgd.json
step b_conv_stock 200 python bench.py --model convnet --impl stock --steps 200 --warmup 30 --json-out gpurun_out/b7_conv_stock.json
echo done
