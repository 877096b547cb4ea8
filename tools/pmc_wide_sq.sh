#!/usr/bin/env bash
# SQ instruction-mix / MFMA-busy passes of the wide int8 prefilter (row n2): two rocprofv3 --pmc passes
# (8 SQ + 1 GRBM counters each: the per-pass limit) over tools/wide_ablate.py CFG B, kernel sq8_wide only.
#   tools/pmc_wide_sq.sh C4 256 [shipped]   → gpurun_out/pmc_sq_<CFG>_<B>[_shipped]_{1,2}/
# (shipped: libosknn.so, the library the bench runs; else the testing build with its clock counters)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-C4}; B=${2:-256}; LIBSEL=${3:-testing}
TL=1; TAG=""
if [[ $LIBSEL == shipped ]]; then TL=0; TAG=_shipped; fi
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  OSK_TESTING_LIB=$TL ABLATE=0 timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex sq8_wide --output-format csv \
      -d gpurun_out/pmc_sq_${CFG}_${B}${TAG}_$i -o run -- python3 tools/wide_ablate.py $CFG $B \
      > gpurun_out/pmc_sq_${CFG}_${B}${TAG}_$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo ok
