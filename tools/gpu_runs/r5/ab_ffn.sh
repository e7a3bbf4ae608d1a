set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5ab
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model bert_large --steps 20 --warmup 8 --json-out gpurun_out/r5ab/bert_fused_$i.json > gpurun_out/r5ab/bert_fused_$i.log 2>&1
  APEX_AMD_GEMM8P=0 timeout -k 10 300 python -u bench.py --model bert_large --steps 20 --warmup 8 --json-out gpurun_out/r5ab/bert_unf_$i.json > gpurun_out/r5ab/bert_unf_$i.log 2>&1
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model gpt2_medium --steps 20 --warmup 8 --json-out gpurun_out/r5ab/gpt2_fused_$i.json > gpurun_out/r5ab/gpt2_fused_$i.log 2>&1
  APEX_AMD_GEMM8P=0 timeout -k 10 300 python -u bench.py --model gpt2_medium --steps 20 --warmup 8 --json-out gpurun_out/r5ab/gpt2_unf_$i.json > gpurun_out/r5ab/gpt2_unf_$i.log 2>&1
done
