set -e
cd /root/repo
run() { timeout -k 10 300 env "$@" python bench.py --steps 5 --warmup 15 --loss-trace > gpurun_out/ay_$1.json 2>> gpurun_out/ay.err; }
run APEX_AMD_NOTHING=1
run APEX_AMD_MT_PERCALL=0
run APEX_AMD_PREP_WEIGHTS=0
run APEX_AMD_REDUCE_ONE=0
run APEX_AMD_WGRAD_STREAM=0
echo ok
