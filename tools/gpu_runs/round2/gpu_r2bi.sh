set -e
cd /root/repo
timeout -k 10 500 bash tools/profile_bench.sh gpt2g 4 --model gpt2_medium --warmup 4
echo ok
