# round 4 box N: is the ResNet-50 step host-bound anywhere? whole-step hipGraph replay
# vs eager (two runs each) and the host-side cProfile of eager steps
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
B="python -u bench.py --steps 20 --warmup 8"
for r in 1 2; do
  timeout -k 10 300 $B --json-out $O/eager_$r.json > $O/eager_$r.log 2>&1
  timeout -k 10 300 $B --graph --json-out $O/graph_$r.json > $O/graph_$r.log 2>&1
done
timeout -k 10 300 python tools/diag/host_profile.py --steps 5 > $O/host_profile.txt 2>&1
echo ok
