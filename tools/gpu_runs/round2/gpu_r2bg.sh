set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/bg_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/bg_smoke.log 2>&1
for m in resnet50 bert_large gpt2_medium; do
  timeout -k 10 300 python bench.py --model $m --loss-trace > gpurun_out/bg_$m.json 2>> gpurun_out/bg.err
done
echo ok
