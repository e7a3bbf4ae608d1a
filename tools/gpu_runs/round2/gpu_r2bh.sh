cd /root/repo
export PYTHONPATH=.
for r in 1 2; do
  for v in fp32 attn ffn; do
    APEX_AMD_DENSE_SIDE=$v timeout -k 10 300 python bench.py --model bert_large > gpurun_out/bh_${v}${r}.json 2>> gpurun_out/bh.err
  done
done
echo ok
