#!/usr/bin/env bash
# Round 6 comparator refresh, ResNet-50: stock PyTorch-ROCm with
# MIOpen find mode (--cudnn-benchmark; the solver search runs silently for minutes, so a
# heartbeat file keeps the call alive) and find mode + TunableOp online tuning, next to
# this framework's headline path, same box.
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6stock
mkdir -p $out
(while true; do date >> $out/heartbeat; sleep 45; done) &
hb=$!
trap 'kill $hb' EXIT
timeout -k 10 840 python -u bench.py --impl stock --cudnn-benchmark --steps 20 --warmup 10 --json-out $out/stock_r50_find.json > $out/stock_r50_find.log 2>&1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=50 \
PYTORCH_TUNABLEOP_FILENAME=$out/stock_r50_tunable.csv \
timeout -k 10 300 python -u bench.py --impl stock --cudnn-benchmark --steps 20 --warmup 10 --json-out $out/stock_r50_find_tunable.json > $out/stock_r50_find_tunable.log 2>&1
timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 --json-out $out/amd_r50_2.json > $out/amd_r50_2.log 2>&1
