set -e
cd /root/repo
timeout -k 10 120 python tools/diag/queue_depth.py > gpurun_out/queue_depth.txt 2>&1
export TMPDIR=/tmp
repo=$(pwd)
cd /tmp
rm -rf /tmp/prof_api2
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --marker-trace --output-format csv -d /tmp/prof_api2 -o run -- python3 $repo/bench.py --steps 4 --warmup 6 > $repo/gpurun_out/prof_api2.log 2>&1
python3 $repo/tools/diag/hip_api_summary.py /tmp/prof_api2 > $repo/gpurun_out/hip_api_r50.md
echo ok
