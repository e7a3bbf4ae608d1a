source tools/gpu_runs/round3/lib.sh
step t_bnbwd 400 $PYT tests/test_conv_bn_bwd_gpu.py
step m_bnbwd 300 python tools/microbench.py conv-bnbwd
step b_r50 300 python bench.py --json-out gpurun_out/b20_r50.json
echo done
