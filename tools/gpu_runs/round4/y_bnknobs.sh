# round 4 box Y: BN elementwise-pass knobs re-checked after the LDS-staged constants
# (rows per thread, rows in flight), ResNet-50, two runs each, same box
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4y
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/def_$r.json > $O/def_$r.log 2>&1
  APEX_AMD_BN_EU=4 timeout -k 10 300 $B --json-out $O/eu4_$r.json > $O/eu4_$r.log 2>&1
  APEX_AMD_BN_TUNING="-1,-1,-1,8,-1,-1" timeout -k 10 300 $B --json-out $O/rpt8_$r.json > $O/rpt8_$r.log 2>&1
  APEX_AMD_BN_TUNING="-1,-1,-1,32,-1,-1" timeout -k 10 300 $B --json-out $O/rpt32_$r.json > $O/rpt32_$r.log 2>&1
  APEX_AMD_BN_TUNING="32,-1,-1,-1,-1,-1" timeout -k 10 300 $B --json-out $O/red32_$r.json > $O/red32_$r.log 2>&1
done
echo ok
