# round 4 box Q: BERT-large host side - host time per step vs GPU time, and every
# host<->device sync inside one step (torch sync-debug mode)
set -e
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 300 python tools/diag/host_profile.py --model bert_large --steps 5 > $O/host_bert.txt 2>&1
timeout -k 10 300 python tools/diag/find_syncs.py --model bert_large > $O/syncs_bert.txt 2>&1
timeout -k 10 300 python tools/diag/host_profile.py --model gpt2_medium --steps 5 > $O/host_gpt2.txt 2>&1
echo ok
