# round 6: sq8_wide_rows COSINE mismatch diagnostics
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'cmd:300:debug_rows.log:python -u tools/debug_rows.py'
