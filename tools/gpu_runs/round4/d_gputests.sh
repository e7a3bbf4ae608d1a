# round 4 box D: the whole GPU suite on the current tree
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/gpu_tests.log 2>&1
echo ok
