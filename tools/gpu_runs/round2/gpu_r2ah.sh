set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest tests/test_embedding_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/emb_tests.log 2>&1
for m in bert_large gpt2_medium; do
  APEX_AMD_SYNCFREE_EMB=0 timeout -k 10 300 python bench.py --model $m > gpurun_out/emb_off_$m.json 2>> gpurun_out/emb.err
  timeout -k 10 300 python bench.py --model $m > gpurun_out/emb_on_$m.json 2>> gpurun_out/emb.err
  APEX_AMD_SYNCFREE_EMB=0 timeout -k 10 300 python bench.py --model $m > gpurun_out/emb_off2_$m.json 2>> gpurun_out/emb.err
  timeout -k 10 300 python bench.py --model $m > gpurun_out/emb_on2_$m.json 2>> gpurun_out/emb.err
done
timeout -k 10 500 bash tools/profile_bench.sh bert2 4 --model bert_large --warmup 4
echo ok
