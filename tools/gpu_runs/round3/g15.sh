source tools/gpu_runs/round3/lib.sh
step d_ddpstats 600 python tools/diag/ddp_stats_diff.py
echo done
