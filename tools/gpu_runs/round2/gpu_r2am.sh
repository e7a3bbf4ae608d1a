set -e
cd /root/repo
for m in bert_large gpt2_medium; do
  for r in 1 2; do
    APEX_AMD_MT_PERCALL=0 APEX_AMD_SYNCFREE_EMB=0 timeout -k 10 300 python bench.py --model $m > gpurun_out/am_old${r}_$m.json 2>> gpurun_out/am.err
    timeout -k 10 300 python bench.py --model $m > gpurun_out/am_new${r}_$m.json 2>> gpurun_out/am.err
  done
done
for r in 1 2; do
  APEX_AMD_MT_PERCALL=0 timeout -k 10 300 python bench.py > gpurun_out/am_old${r}_resnet50.json 2>> gpurun_out/am.err
  timeout -k 10 300 python bench.py > gpurun_out/am_new${r}_resnet50.json 2>> gpurun_out/am.err
done
echo ok
