set -e
cd /root/repo
mkdir -p gpurun_out
rc=0
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_amp_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_h.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --model bert_large --steps 10 --warmup 5 > gpurun_out/bench_bert.json 2> gpurun_out/bench_bert.log
APEX_AMD_LT_GELU=0 timeout -k 10 300 python bench.py --model bert_large --steps 10 --warmup 5 > gpurun_out/bench_bert_nolt.json 2>> gpurun_out/bench_bert.log
timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 5 > gpurun_out/bench_gpt2.json 2> gpurun_out/bench_gpt2.log
APEX_AMD_LT_GELU=0 timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 5 --materialize-master-grads > gpurun_out/bench_gpt2_old.json 2>> gpurun_out/bench_gpt2.log
echo "done tests_rc=$rc"
