set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python tools/diag/host_profile.py --model bert_large --steps 5 > gpurun_out/host_bert2.txt 2>&1
for m in bert_large gpt2_medium; do
  timeout -k 10 300 python bench.py --model $m > gpurun_out/al_$m.json 2>> gpurun_out/al.err
  timeout -k 10 300 python bench.py --model $m > gpurun_out/al2_$m.json 2>> gpurun_out/al.err
done
timeout -k 10 500 bash tools/profile_bench.sh bert5 4 --model bert_large --warmup 4
echo ok
