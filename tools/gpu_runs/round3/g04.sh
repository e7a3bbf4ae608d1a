source tools/gpu_runs/round3/lib.sh
step d_stats 200 python tools/diag/bn_stats_diff.py 16 128
step d_stats_big 200 python tools/diag/bn_stats_diff.py 64 224
echo done
