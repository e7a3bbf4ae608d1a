# round 4 box M: CU-partitioned weight-gradient side stream (APEX_AMD_WGRAD_STREAM_CUS =
# quarters of every XCD's CUs) - GPT-2 (fp32 dense wgrads on the side stream) and ResNet-50
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ddp_gpu.py -k "side_stream" > $O/tests.log 2>&1
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_def_$r.json > $O/gpt2_def_$r.log 2>&1
  for q in 1 2 3; do
    APEX_AMD_WGRAD_STREAM_CUS=$q timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_q${q}_$r.json > $O/gpt2_q${q}_$r.log 2>&1
  done
  timeout -k 10 300 $B --json-out $O/r50_def_$r.json > $O/r50_def_$r.log 2>&1
  for q in 2 3; do
    APEX_AMD_WGRAD_STREAM_CUS=$q timeout -k 10 300 $B --json-out $O/r50_q${q}_$r.json > $O/r50_q${q}_$r.log 2>&1
  done
done
echo ok
