# round 4 box P: attention tests incl. the addressing-variant bitwise test, and the
# native-call microbench with its warm-up (variants read per launch)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_attention_gpu.py > $O/tests.log 2>&1
timeout -k 10 300 python -u tools/microbench.py attn --quick > $O/mb.txt 2>&1
echo ok
