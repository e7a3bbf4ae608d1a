set -e
cd /root/repo
mkdir -p gpurun_out
rc=0
timeout -k 10 600 python -u -m pytest tests/test_ddp_gpu.py tests/test_convergence_gpu.py tests/test_kernels_gpu.py -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "concatenated or resnet18 or maxpool or gelu or syncbn" > gpurun_out/gputests_j.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_r50.json 2> gpurun_out/bench_r50.log
timeout -k 10 400 bash tools/profile_bench.sh r50 8 --warmup 4
echo "done tests_rc=$rc"
