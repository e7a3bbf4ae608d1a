#!/usr/bin/env bash
# LayerNorm backward with one LDS partial row set: tests, per-call bench (new vs ab_old),
# then GPT-2-medium / BERT-large same-box A/B
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6ln
rm -rf $out && mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_bias_handoff_gpu.py tests/test_kernels_gpu.py -k "norm or join or handoff" > $out/tests.log 2>&1
echo tests done
timeout -k 10 120 python -u tools/diag/ln_bwd_bench.py > $out/ln_new.md 2>&1
AB_ROOT=ab_old timeout -k 10 120 python -u tools/diag/ln_bwd_bench.py > $out/ln_old.md 2>&1
for m in gpt2_medium bert_large; do
  for i in 1 2; do
    timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 8 --json-out $out/${m}_new_$i.json > $out/${m}_new_$i.log 2>&1
    timeout -k 10 300 python -u ab_old/bench.py --model $m --steps 20 --warmup 8 --json-out $out/${m}_old_$i.json > $out/${m}_old_$i.log 2>&1
  done
done
