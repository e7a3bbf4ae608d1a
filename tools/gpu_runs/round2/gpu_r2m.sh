set -e
cd /root/repo
mkdir -p gpurun_out
rc=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "conv1x1 or resnet50_fused" > gpurun_out/gputests_m.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_r50.json 2> gpurun_out/bench_r50.log
APEX_AMD_OWN1X1=0 timeout -k 10 300 python bench.py > gpurun_out/bench_r50_noown.json 2>> gpurun_out/bench_r50.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r50b.json 2>> gpurun_out/bench_r50.log
APEX_AMD_OWN1X1=0 timeout -k 10 300 python bench.py > gpurun_out/bench_r50_noownb.json 2>> gpurun_out/bench_r50.log
echo "done tests_rc=$rc"
