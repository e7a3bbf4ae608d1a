set -e
cd /root/repo
mkdir -p gpurun_out
rc=0
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_amp_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "gelu_hipblaslt or mlp or resnet50_fused or bert or gpt2 or folded or overflow or trajectory" > gpurun_out/gputests_f.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --model bert_large --steps 10 --warmup 5 > gpurun_out/bench_bert.json 2> gpurun_out/bench_bert.log
APEX_AMD_LT_GELU=0 timeout -k 10 300 python bench.py --model bert_large --steps 10 --warmup 5 > gpurun_out/bench_bert_nolt.json 2>> gpurun_out/bench_bert.log
timeout -k 10 400 bash tools/profile_bench.sh bert 4 --model bert_large --warmup 3
echo "done tests_rc=$rc"
