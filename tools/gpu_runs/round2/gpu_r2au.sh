set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_final2.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final2.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/f2_resnet50.json 2> gpurun_out/f2.err
timeout -k 10 300 python bench.py --graph > gpurun_out/f2_resnet50_graph.json 2>> gpurun_out/f2.err
timeout -k 10 300 python bench.py --model bert_large > gpurun_out/f2_bert_large.json 2>> gpurun_out/f2.err
timeout -k 10 300 python bench.py --model gpt2_medium > gpurun_out/f2_gpt2_medium.json 2>> gpurun_out/f2.err
timeout -k 10 300 python bench.py --impl stock > gpurun_out/f2_resnet50_stock.json 2>> gpurun_out/f2.err
echo ok
