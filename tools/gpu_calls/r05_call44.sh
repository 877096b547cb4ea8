# LDS occupancy and latency of the wide kernel (C4 b256): one SQ pass of LDS counters
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
ABLATE=0 timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex sq8_wide --output-format csv \
    -d gpurun_out/pmc_lds_C4 -o run -- python3 tools/wide_ablate.py C4 256 > gpurun_out/pmc_lds_C4.log 2>&1 && echo ok
