# round 6: sq8_wide_rows cost split at C4 b256 / C2 b256 (testing build): full, no slow path (4), MFMAs only (8),
# streaming only (1)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'cmd:400:ablate_c4_rows.log:ABLATE=0,4,8,1 python -u tools/wide_ablate.py C4 256' \
  'cmd:400:ablate_c2_rows.log:ABLATE=0,4,8,1 python -u tools/wide_ablate.py C2 256'
