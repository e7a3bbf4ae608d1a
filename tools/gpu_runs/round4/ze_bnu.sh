# round 4 box ZE: rows in flight of the BN read-only reductions (APEX_AMD_BN_U =
# "stats,reduce"; default 4,2): reduce_k measured 2.15 TB/s in profiles/r4/zd
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4ze
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/def_$r.json > $O/def_$r.log 2>&1
  APEX_AMD_BN_U="4,4" timeout -k 10 300 $B --json-out $O/u44_$r.json > $O/u44_$r.log 2>&1
  APEX_AMD_BN_U="8,4" timeout -k 10 300 $B --json-out $O/u84_$r.json > $O/u84_$r.log 2>&1
  APEX_AMD_BN_U="4,8" timeout -k 10 300 $B --json-out $O/u48_$r.json > $O/u48_$r.log 2>&1
done
echo ok
