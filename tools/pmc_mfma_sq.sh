#!/usr/bin/env bash
# SQ instruction-mix / MFMA-busy passes of sq8_mfma (the 32-query int8 MFMA prefilter) at C3 / C4 b32: two
# rocprofv3 --pmc passes (8 SQ + 1 GRBM counters each) over tools/bench_configs.py, kernel sq8_mfma only.
#   tools/pmc_mfma_sq.sh C4 → gpurun_out/pmc_mfma_<CFG>_{1,2}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-C4}
LC=$(echo $CFG | tr 'A-Z' 'a-z')
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex sq8_mfma --output-format csv \
      -d gpurun_out/pmc_mfma_${CFG}_$i -o run -- python3 tools/bench_configs.py --only $CFG --${LC}-batches 32 --steps 4 \
      > gpurun_out/pmc_mfma_${CFG}_$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo ok
