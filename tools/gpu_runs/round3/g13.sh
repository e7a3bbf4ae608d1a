source tools/gpu_runs/round3/lib.sh
step t_all 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider
echo done
