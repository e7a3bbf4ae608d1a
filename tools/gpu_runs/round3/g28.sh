source tools/gpu_runs/round3/lib.sh
step p_fc 500 bash tools/profile_bench.sh r50fc 6 --warmup 4 --force-collectives
echo done
