set -e
cd /root/repo
export PYTHONPATH=.
timeout -k 10 300 python tools/microbench.py wgrad-o1 > gpurun_out/mb_wgrad_o1.txt 2>&1
TORCH_PROF_ROWS=250 timeout -k 10 300 python tools/torch_prof.py > gpurun_out/torch_prof_r50.txt 2>&1
TORCH_PROF_ROWS=120 timeout -k 10 300 python tools/torch_prof.py --model bert_large > gpurun_out/torch_prof_bert.txt 2>&1
echo done
