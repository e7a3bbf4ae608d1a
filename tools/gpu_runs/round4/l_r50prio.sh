# round 4 box L: ResNet-50 stream-priority / side-stream lag re-checks (plain runs)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/def_$r.json > $O/def_$r.log 2>&1
  timeout -k 10 300 $B --main-stream-priority high --json-out $O/mainhi_$r.json > $O/mainhi_$r.log 2>&1
  APEX_AMD_WGRAD_LAG=4 timeout -k 10 300 $B --json-out $O/lag4_$r.json > $O/lag4_$r.log 2>&1
  APEX_AMD_WGRAD_LAG=8 timeout -k 10 300 $B --json-out $O/lag8_$r.json > $O/lag8_$r.log 2>&1
done
echo ok
