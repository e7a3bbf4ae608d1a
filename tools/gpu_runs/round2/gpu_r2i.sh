set -e
cd /root/repo
mkdir -p gpurun_out
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_i.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
PYTHONPATH=. timeout -k 10 120 python -u tools/diag/gelu_epilogue.py > gpurun_out/gelu_epilogue.txt 2>&1
timeout -k 10 300 python bench.py --model bert_large --steps 10 --warmup 5 > gpurun_out/bench_bert.json 2> gpurun_out/bench_bert.log
timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 5 > gpurun_out/bench_gpt2.json 2> gpurun_out/bench_gpt2.log
timeout -k 10 400 bash tools/profile_bench.sh bert 4 --model bert_large --warmup 3
timeout -k 10 400 bash tools/profile_bench.sh gpt2 4 --model gpt2_medium --warmup 3
echo "done tests_rc=$rc"
