source tools/gpu_runs/round3/lib.sh
step t_ln 600 $PYT tests/test_kernels_gpu.py -k "ln or layer_norm or LayerNorm or join" 
step t_models 600 $PYT tests/test_models_gpu.py -k "gpt2 or bert"
step t_guard 400 $PYT tests/test_amp_guard_gpu.py
step b_gpt2 400 python bench.py --model gpt2_medium --json-out gpurun_out/b9_gpt2.json
step b_gpt2_1024 400 env APEX_AMD_LN_BWD_BLOCKS=1024 python bench.py --model gpt2_medium --json-out gpurun_out/b9_gpt2_1024.json
step b_bert 400 python bench.py --model bert_large --json-out gpurun_out/b9_bert.json
step p_gpt2 500 bash tools/profile_bench.sh gpt2ln 4 --model gpt2_medium --warmup 4
echo done
