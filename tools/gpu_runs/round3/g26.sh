source tools/gpu_runs/round3/lib.sh
step t_all 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider
step b_r50 300 python bench.py --json-out gpurun_out/b26_r50.json
step b_r50b 300 python bench.py --json-out gpurun_out/b26_r50b.json
step b_gpt2 300 python bench.py --model gpt2_medium --json-out gpurun_out/b26_gpt2.json
echo done
