set -e
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem" > gpurun_out/stem_test.log 2>&1
rm -f gpurun_out/stem_mb2.log
bash tools/stem_gpu2.sh
