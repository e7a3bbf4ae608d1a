source tools/gpu_runs/round3/lib.sh
step h_fc 300 python tools/diag/host_profile.py --force-collectives --steps 10
step h_std 300 python tools/diag/host_profile.py --steps 10
echo done
