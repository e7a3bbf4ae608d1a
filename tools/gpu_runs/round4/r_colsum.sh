# round 4 box R: bias-gradient stage 2 with 16 columns x 16 split lanes per block
# (default) vs the wide 64 x 4 form (APEX_AMD_COLSUM_FINAL=64): dense / MLP tests and
# GPT-2-medium / BERT-large steps, two runs each
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "bias_grad or mlp or dense or gelu" tests/test_determinism_gpu.py tests/test_gemm8p_gpu.py > $O/tests.log 2>&1
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_def_$r.json > $O/gpt2_def_$r.log 2>&1
  APEX_AMD_COLSUM_FINAL=64 timeout -k 10 300 $B --model gpt2_medium --json-out $O/gpt2_w64_$r.json > $O/gpt2_w64_$r.log 2>&1
  timeout -k 10 300 $B --model bert_large --json-out $O/bert_def_$r.json > $O/bert_def_$r.log 2>&1
  APEX_AMD_COLSUM_FINAL=64 timeout -k 10 300 $B --model bert_large --json-out $O/bert_w64_$r.json > $O/bert_w64_$r.log 2>&1
done
echo ok
