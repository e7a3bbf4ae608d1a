set -e
cd /root/repo
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 300 python -u tools/microbench.py conv-bm > gpurun_out/mb_conv_bm.txt 2>&1
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gputests_o.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
timeout -k 10 300 python bench.py --impl stock > gpurun_out/bench_stock.json 2> gpurun_out/bench_stock.log
echo "done tests_rc=$rc"
