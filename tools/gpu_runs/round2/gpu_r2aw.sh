set -e
cd /root/repo
timeout -k 10 500 bash tools/profile_bench.sh r50f 8 --warmup 6
timeout -k 10 300 python bench.py > gpurun_out/aw_resnet50.json 2> gpurun_out/aw.err
echo ok
