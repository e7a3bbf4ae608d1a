source tools/gpu_runs/round3/lib.sh
step t_graph 300 $PYT tests/test_graph_gpu.py
step m_lnj 120 python tools/microbench.py ln-join
step m_lnj512 120 env APEX_AMD_LN_BWD_BLOCKS=512 python tools/microbench.py ln-join
step m_lnj2048 120 env APEX_AMD_LN_BWD_BLOCKS=2048 python tools/microbench.py ln-join
step bg_bert 300 python bench.py --model bert_large --graph --json-out gpurun_out/b11_bert_graph.json
step bg_gpt2 300 python bench.py --model gpt2_medium --graph --json-out gpurun_out/b11_gpt2_graph.json
step bg_r50 300 python bench.py --graph --json-out gpurun_out/b11_r50_graph.json
echo done
