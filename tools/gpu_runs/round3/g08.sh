source tools/gpu_runs/round3/lib.sh
step d_guard 120 python tools/diag/guard_diff.py
step mb_stats 300 python tools/microbench.py conv1x1-stats
step b_stats 300 python bench.py --json-out gpurun_out/b8_stats.json
echo done
