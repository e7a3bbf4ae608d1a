set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ac.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_ac.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_ac.json 2> gpurun_out/bench_ac.err
timeout -k 10 300 python bench.py > gpurun_out/bench_ac2.json 2>> gpurun_out/bench_ac.err
echo done
