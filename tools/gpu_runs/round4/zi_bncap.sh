# round 4 box ZI: BN reduction grid after the branch-free reduce_k (cap 2048 / 4096,
# 16 rows per thread), ResNet-50 two runs each, same box
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4zi
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/def_$r.json > $O/def_$r.log 2>&1
  APEX_AMD_BN_TUNING="-1,2048,-1,-1,-1,-1" timeout -k 10 300 $B --json-out $O/cap2k_$r.json > $O/cap2k_$r.log 2>&1
  APEX_AMD_BN_TUNING="-1,4096,-1,-1,-1,-1" timeout -k 10 300 $B --json-out $O/cap4k_$r.json > $O/cap4k_$r.log 2>&1
  APEX_AMD_BN_TUNING="16,2048,-1,-1,-1,-1" timeout -k 10 300 $B --json-out $O/r16c2k_$r.json > $O/r16c2k_$r.log 2>&1
done
echo ok
