# round 4 box Z: BN grid knobs, second pass (rows per thread of the elementwise passes
# 8 / 4, reduction rows per thread 32 / 16), ResNet-50, two runs each, same box
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/def_$r.json > $O/def_$r.log 2>&1
  APEX_AMD_BN_TUNING="-1,-1,-1,8,-1,-1" timeout -k 10 300 $B --json-out $O/rpt8_$r.json > $O/rpt8_$r.log 2>&1
  APEX_AMD_BN_TUNING="-1,-1,-1,4,-1,-1" timeout -k 10 300 $B --json-out $O/rpt4_$r.json > $O/rpt4_$r.log 2>&1
  APEX_AMD_BN_TUNING="32,-1,-1,8,-1,-1" timeout -k 10 300 $B --json-out $O/r32e8_$r.json > $O/r32e8_$r.log 2>&1
  APEX_AMD_BN_TUNING="16,-1,-1,8,-1,-1" timeout -k 10 300 $B --json-out $O/r16e8_$r.json > $O/r16e8_$r.log 2>&1
done
echo ok
