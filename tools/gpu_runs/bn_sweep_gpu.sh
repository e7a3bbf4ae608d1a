set -e
cd /root/repo
for t in "-1,-1,-1,-1,-1,-1" "-1,-1,-1,-1,-1,2048" "-1,-1,1024,-1,-1,-1" "-1,-1,1024,-1,-1,2048" "-1,-1,-1,8,-1,-1" "32,-1,-1,-1,-1,-1"; do
  APEX_AMD_BN_TUNING="$t" timeout -k 10 200 python -u bench.py --steps 30 --warmup 10 > gpurun_out/bn_sweep.log 2>&1
  echo "$t $(tail -1 gpurun_out/bn_sweep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/bn_sweep.txt
done
