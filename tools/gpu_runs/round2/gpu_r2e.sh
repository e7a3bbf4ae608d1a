set -e
cd /root/repo
mkdir -p gpurun_out
rc=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_amp_gpu.py tests/test_models_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_e.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 python -u tools/diag/gelu_epilogue.py > gpurun_out/gelu_epilogue.txt 2>&1
timeout -k 10 300 python bench.py --model bert_large --steps 10 --warmup 5 > gpurun_out/bench_bert.json 2> gpurun_out/bench_bert.log
echo "done tests_rc=$rc"
