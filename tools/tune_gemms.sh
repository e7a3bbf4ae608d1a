#!/usr/bin/env bash
# Tune the library GEMMs of bench.py's training steps in situ with PyTorch
# TunableOp (rocBLAS + hipBLASLt solutions timed per shape) and write the
# selections to gpurun_out/tuning/<model>.csv; commit them as tuning/<model>.csv,
# which bench.py (--gemm-tuning auto) then loads read-only.  Run on an MI355X:
#   tools/tune_gemms.sh resnet50 bert_large gpt2_medium
# Each model: one short bench run with tuning on (every GEMM shape of the step
# hits the tuner during warmup), then an A/B of tuned vs untuned.
set -eu
repo="$(cd "$(dirname "$0")/.." && pwd)"
cd "$repo"
out=gpurun_out/tuning
mkdir -p "$out"
# the tuner runs silently for minutes: keep a heartbeat file fresh
( while true; do date >> gpurun_out/heartbeat.txt; sleep 30; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-100}
export PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=${TUNE_ITERS:-100}
# rotate operands through a 512 MB pool so no candidate is timed L2/MALL-hot
export PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=${TUNE_ROTATE_MB:-512}
for m in "$@"; do
  rm -f "$out/$m"*.csv
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
  PYTORCH_TUNABLEOP_FILENAME="$out/$m%d.csv" \
    timeout -k 10 900 python bench.py --model "$m" --gemm-tuning off --steps 2 --warmup 2 \
      > "$out/${m}_tuning.json" 2> "$out/${m}_tuning.log"
  cp "$out/${m}0.csv" "$out/$m.csv"
  timeout -k 10 300 python bench.py --model "$m" --gemm-tuning off > "$out/${m}_off.json" \
    2> "$out/${m}_off.log"
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME="$out/$m%d.csv" \
    timeout -k 10 300 python bench.py --model "$m" > "$out/${m}_tuned.json" 2> "$out/${m}_tuned.log"
done
echo tuned "$@"
