# round 4 box E: rocprofv3 kernel tables of the current tree (plain runs and ResNet-50
# under forced collectives) -> gpurun_out/prof_*.md, copied to profiles/ by hand
set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 240 bash tools/profile_bench.sh r50 10 --warmup 5
timeout -k 10 240 bash tools/profile_bench.sh r50fc 10 --warmup 5 --force-collectives
timeout -k 10 240 bash tools/profile_bench.sh bert 10 --warmup 5 --model bert_large
timeout -k 10 240 bash tools/profile_bench.sh gpt2 10 --warmup 5 --model gpt2_medium
timeout -k 10 240 bash tools/profile_bench.sh gpt2fc 10 --warmup 5 --model gpt2_medium --force-collectives
echo ok
