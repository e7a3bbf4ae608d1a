set -e
cd /root/repo
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 300 python -u tools/microbench.py conv1x1-own > gpurun_out/mb_conv1x1_own.txt 2>&1
echo done
