set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 400 bash tools/profile_bench.sh r50 8 --warmup 6
timeout -k 10 300 python tools/torch_prof.py > gpurun_out/torch_prof_r50.txt 2>&1
echo done
