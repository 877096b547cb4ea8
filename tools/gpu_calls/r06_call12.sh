# round 6: evidence for the shipped library — kernel trace + FETCH/WRITE of C4 b1024 and C2 b256, and the SQ
# counter passes (MFMA busy, instruction mix) of the shipped wide kernels at C4 b256 (sq8_wide_rows) and C3 b256
# (sq8_wide, KS = 12)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh \
  'cmd:700:prof_c4.log:bash tools/prof_wide.sh r06_c4 "--only C4 --c4-batches 1024 --steps 3"' \
  'cmd:400:prof_c2.log:bash tools/prof_wide.sh r06_c2 "--only C2 --c2-batches 256 --steps 5"' \
  'cmd:600:pmc_sq_c4.log:bash tools/pmc_wide_sq.sh C4 256 shipped' \
  'cmd:600:pmc_sq_c3.log:bash tools/pmc_wide_sq.sh C3 256 shipped' \
  'cmd:120:pmc_sq_sum.log:python3 tools/pmc_sq_summary.py gpurun_out/pmc_sq_C4_256_shipped.json gpurun_out/pmc_sq_C4_256_shipped_1 gpurun_out/pmc_sq_C4_256_shipped_2 shipped && python3 tools/pmc_sq_summary.py gpurun_out/pmc_sq_C3_256_shipped.json gpurun_out/pmc_sq_C3_256_shipped_1 gpurun_out/pmc_sq_C3_256_shipped_2 shipped'
