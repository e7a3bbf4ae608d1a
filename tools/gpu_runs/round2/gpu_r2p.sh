set -e
cd /root/repo
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 300 python -u tools/microbench.py conv-bm > gpurun_out/mb_conv_bm.txt 2>&1
echo done
