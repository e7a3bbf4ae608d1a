set -e
cd /root/repo
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 400 python -u tools/microbench.py bn-u > gpurun_out/mb_bn_u.txt 2>&1
echo done
