source tools/gpu_runs/round3/lib.sh
step b_fc 400 python bench.py --force-collectives --json-out gpurun_out/b27_fc.json
step b_r50 300 python bench.py --json-out gpurun_out/b27_r50.json
step p_r50 400 bash tools/profile_bench.sh r50r3 8 --warmup 4
step t_lamb 200 $PYT tests/test_kernels_gpu.py -k legacy_lamb
echo done
