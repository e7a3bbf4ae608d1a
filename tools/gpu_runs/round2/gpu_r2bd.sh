cd /root/repo
export PYTHONPATH=.
for m in resnet50 bert_large gpt2_medium; do
  timeout -k 10 300 python bench.py --model $m --loss-trace > gpurun_out/bd_on_$m.json 2>> gpurun_out/bd.err
  timeout -k 10 300 python bench.py --model $m --loss-trace --gemm-tuning off > gpurun_out/bd_off_$m.json 2>> gpurun_out/bd.err
done
echo ok
