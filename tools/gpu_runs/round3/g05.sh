source tools/gpu_runs/round3/lib.sh
step t_stats 400 $PYT tests/test_conv_bn_stats_gpu.py
step mb_nb1_0 300 env APEX_AMD_CONV1X1_NB1=0 python tools/microbench.py conv1x1-stats
step mb_nb1_1 300 env APEX_AMD_CONV1X1_NB1=1 python tools/microbench.py conv1x1-stats
step mb_nb1_2 300 env APEX_AMD_CONV1X1_NB1=2 python tools/microbench.py conv1x1-stats
step b_nb0 300 env APEX_AMD_CONV1X1_NB1=0 python bench.py --json-out gpurun_out/b5_nb0.json
step b_nb1 300 env APEX_AMD_CONV1X1_NB1=1 python bench.py --json-out gpurun_out/b5_nb1.json
step b_nb2 300 env APEX_AMD_CONV1X1_NB1=2 python bench.py --json-out gpurun_out/b5_nb2.json
step b_nostats 300 env APEX_AMD_CONV_BN_STATS=0 python bench.py --json-out gpurun_out/b5_nostats.json
echo done
