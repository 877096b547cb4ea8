# round 6: where sq8_mfma (32 queries per launch) spends C3 / C4 b32 — SQ passes and a kernel trace
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'cmd:600:pmc_mfma_c4.log:bash tools/pmc_mfma_sq.sh C4' 'cmd:600:pmc_mfma_c3.log:bash tools/pmc_mfma_sq.sh C3' \
  'cmd:120:pmc_mfma_sum.log:KINDS=pilot,main python3 tools/pmc_sq_summary.py gpurun_out/pmc_mfma_C4.json gpurun_out/pmc_mfma_C4_1 gpurun_out/pmc_mfma_C4_2 C4b32 && KINDS=pilot,main python3 tools/pmc_sq_summary.py gpurun_out/pmc_mfma_C3.json gpurun_out/pmc_mfma_C3_1 gpurun_out/pmc_mfma_C3_2 C3b32' \
  'cmd:400:prof22.log:bash tools/prof_wide.sh r06_b32 "--only C3,C4 --c3-batches 32 --c4-batches 32 --steps 4"' || exit $?
