set -e
cd /root/repo
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 120 python -u tools/diag/lt_probe.py > gpurun_out/lt_probe.txt 2>&1
rc=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "maxpool or resnet50_fused or bn" > gpurun_out/gputests_g.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_r50.json 2> gpurun_out/bench_r50.log
APEX_AMD_FUSE_STEM=0 timeout -k 10 300 python bench.py > gpurun_out/bench_r50_nostem.json 2>> gpurun_out/bench_r50.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r50b.json 2>> gpurun_out/bench_r50.log
echo "done tests_rc=$rc"
