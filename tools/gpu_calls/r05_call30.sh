# where sq8_wide's step time goes after the SGPR descriptors: ablations (results wrong, timing only)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "cmd:300:ablate30_c4.log:ABLATE=0,1,2,3,8,9,64 python -u tools/wide_ablate.py C4 256" \
  "cmd:300:ablate30_c3.log:ABLATE=0,1,2,8,64 python -u tools/wide_ablate.py C3 256"
