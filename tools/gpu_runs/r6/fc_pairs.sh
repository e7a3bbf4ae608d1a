#!/usr/bin/env bash
# plain vs forced 1-rank RCCL collectives (DDP + SyncBN path) for the three models, one box
set -eu
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6fc
mkdir -p $out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29571
for m in resnet50 bert_large gpt2_medium; do
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 8 --json-out $out/${m}_plain.json > $out/${m}_plain.log 2>&1
  timeout -k 10 300 python -u bench.py --model $m --steps 20 --warmup 8 --force-collectives --json-out $out/${m}_fc.json > $out/${m}_fc.log 2>&1
done
