set -e
cd /root/repo
mkdir -p gpurun_out
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests.log 2>&1 || rc=$?
# test failures (1) still allow the measurements; a timeout / crash ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u tools/microbench.py optim > gpurun_out/mb_optim.txt 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
echo "done tests_rc=$rc"
