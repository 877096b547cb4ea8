# round 6: where sq8_wide_rows' time goes at C4 b256 (ablations on the testing build) and a kernel trace +
# FETCH/WRITE passes of C4 b1024 per launch set (pilot, first pass, second pass)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'cmd:400:ablate_c4_rows.log:ABLATE=0,1,2,3 python -u tools/wide_ablate.py C4 256' \
  'cmd:400:ablate_c2_rows.log:ABLATE=0,1,2,3 python -u tools/wide_ablate.py C2 256' \
  'cmd:900:prof_c4.log:bash tools/prof_wide.sh r06a_c4 "--only C4 --c4-batches 1024 --steps 3"' \
  'cmd:120:sets_c4.log:python3 tools/wide_launch_sets.py gpurun_out/r06a_c4 gpurun_out/r06a_c4/wide_launch_sets.json "C4 b1024 sq8_wide_rows" "per 256 queries: 100M rows x (128 B tiled int8 + staged terms)"'
