#!/usr/bin/env bash
# Round 6 comparator refresh for the transformer configs: stock
# PyTorch-ROCm BERT-large / GPT-2-medium (plain and TunableOp online tuning) next to this
# framework's path, same box.
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6stx
mkdir -p $out
(while true; do date >> $out/heartbeat; sleep 45; done) &
hb=$!
trap 'kill $hb' EXIT
for m in bert_large gpt2_medium; do
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 8 --json-out $out/amd_$m.json > $out/amd_$m.log 2>&1
  timeout -k 10 300 python -u bench.py --model $m --impl stock --steps 20 --warmup 8 --json-out $out/stock_$m.json > $out/stock_$m.log 2>&1
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 \
  PYTORCH_TUNABLEOP_FILENAME=$out/stock_${m}_tunable.csv \
  timeout -k 10 500 python -u bench.py --model $m --impl stock --steps 20 --warmup 8 --json-out $out/stock_${m}_tunable.json > $out/stock_${m}_tunable.log 2>&1
done
