# round 4 box ZD: HBM bytes of the BN / pool kernels in a short ResNet-50 run
# (FETCH_SIZE and WRITE_SIZE in separate passes, kernel trace only)
set -e
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 bash tools/diag/run_pmc.sh bench.py tools/diag/bn_bw_pmc.txt --steps 3 --warmup 2
mkdir -p gpurun_out/r4zd
mv gpurun_out/pmc_*.csv gpurun_out/pmc.log gpurun_out/r4zd/
echo ok
