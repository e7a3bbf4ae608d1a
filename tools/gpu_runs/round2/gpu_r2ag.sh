set -e
cd /root/repo
for m in bert_large gpt2_medium resnet50; do
  timeout -k 10 300 python tools/diag/find_syncs.py --model $m > gpurun_out/syncs_$m.txt 2>&1
done
echo ok
