set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python tools/microbench.py bn-eu > gpurun_out/mb_bn_eu2.txt 2>&1
for i in 1 2; do
  APEX_AMD_BN_ELEM_FIXED=1 timeout -k 10 300 python bench.py > gpurun_out/ab_fixed_$i.json 2>> gpurun_out/ab.log
  timeout -k 10 300 python bench.py > gpurun_out/ab_auto_$i.json 2>> gpurun_out/ab.log
done
timeout -k 10 400 bash tools/profile_bench.sh r50 8 --warmup 6
timeout -k 10 400 bash tools/profile_bench.sh bert 4 --warmup 4 --model bert_large
timeout -k 10 400 bash tools/profile_bench.sh gpt2 4 --warmup 4 --model gpt2_medium
echo done
