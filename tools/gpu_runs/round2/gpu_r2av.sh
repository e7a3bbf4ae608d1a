set -e
cd /root/repo
timeout -k 10 500 bash tools/profile_bench.sh bertf 4 --model bert_large --warmup 4
timeout -k 10 500 bash tools/profile_bench.sh gpt2f 4 --model gpt2_medium --warmup 4
echo ok
