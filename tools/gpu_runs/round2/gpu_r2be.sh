set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/be_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/be_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/be_resnet50.json 2> gpurun_out/be.err
timeout -k 10 500 bash tools/profile_bench.sh r50g 8 --warmup 6
echo ok
