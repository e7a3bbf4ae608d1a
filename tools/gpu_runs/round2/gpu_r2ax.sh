set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ax_tests.log 2>&1
for r in 1 2; do
  APEX_AMD_WGRAD_STREAM=0 timeout -k 10 300 python bench.py > gpurun_out/ax_off${r}.json 2>> gpurun_out/ax.err
  timeout -k 10 300 python bench.py > gpurun_out/ax_on${r}.json 2>> gpurun_out/ax.err
done
timeout -k 10 300 python bench.py --loss-trace > gpurun_out/ax_trace_on.json 2>> gpurun_out/ax.err
APEX_AMD_WGRAD_STREAM=0 timeout -k 10 300 python bench.py --loss-trace > gpurun_out/ax_trace_off.json 2>> gpurun_out/ax.err
echo ok
