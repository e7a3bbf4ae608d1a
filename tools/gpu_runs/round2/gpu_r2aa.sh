set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python tools/microbench.py wgrad-dense > gpurun_out/mb_wgrad_dense.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "avg_pool or maxpool or resnet" > gpurun_out/gputests_aa.log 2>&1
for i in 1 2; do
  APEX_AMD_GAP_OFF=1 timeout -k 10 300 python bench.py > gpurun_out/gap_off_$i.json 2>> gpurun_out/gap.log
  timeout -k 10 300 python bench.py > gpurun_out/gap_on_$i.json 2>> gpurun_out/gap.log
done
echo done
