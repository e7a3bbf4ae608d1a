# round 4 box X: rocprofv3 kernel tables of the final tree -> gpurun_out/prof_*.md
set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 240 bash tools/profile_bench.sh r50 10 --warmup 5
timeout -k 10 240 bash tools/profile_bench.sh r50fc 10 --warmup 5 --force-collectives
timeout -k 10 240 bash tools/profile_bench.sh bert 10 --warmup 5 --model bert_large
timeout -k 10 240 bash tools/profile_bench.sh gpt2 10 --warmup 5 --model gpt2_medium
echo ok
