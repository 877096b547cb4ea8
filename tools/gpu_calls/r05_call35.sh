# upper bound of a cheaper enqueue: the wide kernel with its quick tests but no enqueue (ablate 32)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "cmd:300:ablate35_c4.log:ABLATE=0,32,0,32 python -u tools/wide_ablate.py C4 256" \
  "cmd:300:ablate35_c3.log:ABLATE=0,32 python -u tools/wide_ablate.py C3 256"
