set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_ab.log 2>&1
for m in bert_large gpt2_medium; do
  APEX_AMD_DENSE_SPLITK=0 timeout -k 10 300 python bench.py --model $m > gpurun_out/sk_off_$m.json 2>> gpurun_out/sk.log
  timeout -k 10 300 python bench.py --model $m > gpurun_out/sk_on_$m.json 2>> gpurun_out/sk.log
  APEX_AMD_DENSE_SPLITK=0 timeout -k 10 300 python bench.py --model $m > gpurun_out/sk_off2_$m.json 2>> gpurun_out/sk.log
  timeout -k 10 300 python bench.py --model $m > gpurun_out/sk_on2_$m.json 2>> gpurun_out/sk.log
done
echo done
