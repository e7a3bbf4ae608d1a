set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_convergence_gpu.py tests/test_amp_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_d.log 2>&1
timeout -k 10 300 python -u tools/microbench.py optim --wgs 0 2 4 > gpurun_out/mb_optim.txt 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
timeout -k 10 300 python bench.py --model bert_large --steps 10 --warmup 5 > gpurun_out/bench_bert.json 2> gpurun_out/bench_bert.log
timeout -k 10 400 bash tools/profile_bench.sh r50 8 --warmup 4
echo done
