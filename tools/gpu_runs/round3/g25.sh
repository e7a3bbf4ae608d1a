source tools/gpu_runs/round3/lib.sh
step t_mix 600 $PYT tests/test_amp_gpu.py tests/test_ddp_gpu.py tests/test_kernels_gpu.py -k "native_plan or syncbn or two_ranks or side_stream or legacy_lamb"
step b_r50 300 python bench.py --json-out gpurun_out/b25_r50.json
step p_ser 400 env APEX_AMD_WGRAD_STREAM=0 bash tools/profile_bench.sh r50ser3 4 --warmup 4
step p_disp 200 python tools/rocprof_summary.py /tmp/prof_r50ser3 --range timed_steps --steps 4 --top 5 --dispatch-filter "apply_k|backward_k|reduce_k|stats_from|slab_fold|reduce_finalize" --dispatch-out gpurun_out/disp_r50ser3.txt
step b_bert 300 python bench.py --model bert_large --json-out gpurun_out/b25_bert.json
echo done
