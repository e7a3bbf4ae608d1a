set -e
cd /root/repo
export TMPDIR=/tmp
repo=$(pwd)
cd /tmp
rm -rf /tmp/prof_api
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --marker-trace --output-format csv -d /tmp/prof_api -o run -- python3 $repo/bench.py --model bert_large --steps 4 --warmup 4 > $repo/gpurun_out/prof_api.log 2>&1
python3 $repo/tools/diag/hip_api_summary.py /tmp/prof_api > $repo/gpurun_out/hip_api_bert.md
echo ok
