# round 4 box I: the BN-backward dgrad-epilogue size limit re-checked on the 32-deep ring
# (APEX_AMD_CONV_BN_BWD_MAXM: default 16384 output pixels without a residual)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/r50_def_$r.json > $O/r50_def_$r.log 2>&1
  APEX_AMD_CONV_BN_BWD_MAXM=200000 timeout -k 10 300 $B --json-out $O/r50_m200k_$r.json > $O/r50_m200k_$r.log 2>&1
  APEX_AMD_CONV_BN_BWD_MAXM=100000000 timeout -k 10 300 $B --json-out $O/r50_mall_$r.json > $O/r50_mall_$r.log 2>&1
done
echo ok
