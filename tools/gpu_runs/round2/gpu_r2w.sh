set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python tools/microbench.py bn-eu > gpurun_out/mb_bn_eu.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_w.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_w.log 2>&1
echo done
