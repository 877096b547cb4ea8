set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "cmd:400:wide_abl2.log:ABLATE=0,8,32,40 python -u tools/wide_ablate.py C4 256 && ABLATE=0,8,32,40 python -u tools/wide_ablate.py C3 256"
