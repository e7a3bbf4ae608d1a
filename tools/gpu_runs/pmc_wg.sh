set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_wg
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_wg/a -o run -- python3 tools/prof_wgrad.py 0 1 > gpurun_out/pmc_wg/a.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_wg/t -o run -- python3 tools/prof_wgrad.py 0 1 > gpurun_out/pmc_wg/t.log 2>&1
echo done
