set -e
cd /root/repo
bash tools/tune_gemms.sh resnet50 bert_large gpt2_medium
timeout -k 10 300 python bench.py --model bert_large --graph --gemm-tuning off > gpurun_out/bert_graph.json 2> gpurun_out/bert_graph.log
echo done
