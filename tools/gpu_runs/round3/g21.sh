source tools/gpu_runs/round3/lib.sh
step t_bnbwd 400 $PYT tests/test_conv_bn_bwd_gpu.py
step b_r50 300 python bench.py --json-out gpurun_out/b21_r50.json
step b_r50off 300 env APEX_AMD_CONV_BN_BWD=0 python bench.py --json-out gpurun_out/b21_r50off.json
step b_r50b 300 python bench.py --json-out gpurun_out/b21_r50b.json
echo done
