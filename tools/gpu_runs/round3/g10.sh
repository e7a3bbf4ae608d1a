source tools/gpu_runs/round3/lib.sh
step t_ln 600 $PYT tests/test_kernels_gpu.py -k "ln or layer_norm or LayerNorm or join or bias or gelu or colsum"
step b_gpt2 400 python bench.py --model gpt2_medium --json-out gpurun_out/b10_gpt2.json
step b_bert 400 python bench.py --model bert_large --json-out gpurun_out/b10_bert.json
step b_r50 300 python bench.py --json-out gpurun_out/b10_r50.json
step p_gpt2 500 bash tools/profile_bench.sh gpt2ln2 4 --model gpt2_medium --warmup 4
step d_graph 400 python tools/diag/bert_graph.py
echo done
