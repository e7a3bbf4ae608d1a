set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_r50.json 2> gpurun_out/bench_r50.log
timeout -k 10 400 bash tools/profile_bench.sh r50 8 --warmup 4
echo done
