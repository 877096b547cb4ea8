set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "cmd:900:c3o.log:python -u tools/bench_configs.py --only C3o --steps 20"
