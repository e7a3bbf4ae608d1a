set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_v.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_v.log 2>&1
timeout -k 10 400 bash tools/profile_bench.sh r50 8 --warmup 6
timeout -k 10 400 bash tools/profile_bench.sh bert 4 --warmup 4 --model bert_large
timeout -k 10 400 bash tools/profile_bench.sh gpt2 4 --warmup 4 --model gpt2_medium
echo done
