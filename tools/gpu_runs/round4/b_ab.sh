# round 4 box B: DDP / amp GPU tests after lazy zeroing + tapered buckets, in-model A/Bs
# (64-channel strip-ring wgrad, side-stream priority / DDP side stream), GPT-2 forced
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm8p_gpu.py > $O/gemm8p_tests.log 2>&1
timeout -k 10 300 python -u tools/gemm8p_bench.py > $O/gemm8p_bench.md 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_ddp_gpu.py tests/test_amp_gpu.py tests/test_graph_gpu.py tests/test_conv_bn_bwd_gpu.py \
  tests/test_models_gpu.py > $O/tests.log 2>&1
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  APEX_AMD_WGRAD64=1 timeout -k 10 300 $B --json-out $O/r50_w64_$r.json > $O/r50_w64_$r.log 2>&1
  APEX_AMD_WGRAD64=0 timeout -k 10 300 $B --json-out $O/r50_tap_$r.json > $O/r50_tap_$r.log 2>&1
  APEX_AMD_WGRAD_STREAM_PRIO=high timeout -k 10 300 $B --json-out $O/r50_prio_$r.json > $O/r50_prio_$r.log 2>&1
  APEX_AMD_CONV_PAIR_S2=0 timeout -k 10 300 $B --json-out $O/r50_nopair_$r.json > $O/r50_nopair_$r.log 2>&1
done
for r in 1 2; do
  timeout -k 10 300 $B --force-collectives --json-out $O/fc_$r.json > $O/fc_$r.log 2>&1
  APEX_AMD_WGRAD_STREAM_DDP=1 timeout -k 10 300 $B --force-collectives --json-out $O/fc_side_$r.json > $O/fc_side_$r.log 2>&1
  APEX_AMD_WGRAD_STREAM_DDP=1 APEX_AMD_WGRAD_STREAM_PRIO=high timeout -k 10 300 $B --force-collectives --json-out $O/fc_sidep_$r.json > $O/fc_sidep_$r.log 2>&1
done
timeout -k 10 300 $B --model gpt2_medium --force-collectives --json-out $O/gpt2_fc.json > $O/gpt2_fc.log 2>&1
timeout -k 10 300 $B --model bert_large --json-out $O/bert.json > $O/bert.log 2>&1
echo ok
