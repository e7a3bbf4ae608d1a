set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final_resnet50.json 2> gpurun_out/final.err
timeout -k 10 300 python bench.py --model bert_large > gpurun_out/final_bert_large.json 2>> gpurun_out/final.err
timeout -k 10 300 python bench.py --model gpt2_medium > gpurun_out/final_gpt2_medium.json 2>> gpurun_out/final.err
timeout -k 10 500 bash tools/profile_bench.sh r50final 8 --warmup 6
echo ok
