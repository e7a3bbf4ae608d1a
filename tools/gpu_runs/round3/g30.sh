source tools/gpu_runs/round3/lib.sh
step t_ddp 600 $PYT tests/test_ddp_gpu.py
step b_fc 400 python bench.py --force-collectives --json-out gpurun_out/b30_fc.json
step b_r50 300 python bench.py --json-out gpurun_out/b30_r50.json
step p_fc 500 bash tools/profile_bench.sh r50fc2 6 --warmup 4 --force-collectives
echo done
