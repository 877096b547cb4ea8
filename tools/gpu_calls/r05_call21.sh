set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh smoke "bench" prof pmc
