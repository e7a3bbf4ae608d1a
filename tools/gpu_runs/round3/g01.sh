source tools/gpu_runs/round3/lib.sh
step t_syncbn_forced 300 $PYT tests/test_ddp_gpu.py -k "forced or race"
step t_emb_det 400 $PYT tests/test_embedding_gpu.py tests/test_determinism_gpu.py
step t_examples 600 $PYT tests/test_examples_gpu.py
PYTORCH_TUNABLEOP_VERBOSE=3 PYTORCH_TUNABLEOP_VERBOSE_FILENAME=gpurun_out/tunable_verbose.log \
  step v_tuned 300 python tools/diag/tuned_gemm_validate.py resnet50 --out gpurun_out/tuned_r50.json
step t_tuned 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gemm_tuning_gpu.py
step b_r50 300 python bench.py --json-out gpurun_out/b_r50.json
step b_r50_forced 300 python bench.py --force-collectives --json-out gpurun_out/b_r50_forced.json
step b_conv_sgd 200 python bench.py --model convnet --steps 200 --warmup 30 --json-out gpurun_out/b_conv_sgd.json
step b_conv_fused 200 python bench.py --model convnet --steps 200 --warmup 30 --convnet-optimizer fused --json-out gpurun_out/b_conv_fused.json
step b_conv_stock 200 python bench.py --model convnet --impl stock --steps 200 --warmup 30 --json-out gpurun_out/b_conv_stock.json
step p_r50_serial 400 env APEX_AMD_WGRAD_STREAM=0 bash tools/profile_bench.sh r50serial 8 --warmup 4
echo done
