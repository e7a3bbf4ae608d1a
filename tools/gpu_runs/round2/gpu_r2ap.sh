set -e
cd /root/repo
export TMPDIR=/tmp
repo=$(pwd)
cd /tmp
rm -rf /tmp/prof_api3
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --marker-trace --output-format csv -d /tmp/prof_api3 -o run -- python3 $repo/bench.py --steps 4 --warmup 6 > $repo/gpurun_out/prof_api3.log 2>&1
python3 $repo/tools/diag/hip_api_summary.py /tmp/prof_api3 > $repo/gpurun_out/hip_api_r50b.md
head -3 /tmp/prof_api3/*/*hip_api_trace.csv > $repo/gpurun_out/hip_api_cols.txt 2>&1 || true
head -3 /tmp/prof_api3/*/*kernel_trace.csv >> $repo/gpurun_out/hip_api_cols.txt 2>&1 || true
echo ok
