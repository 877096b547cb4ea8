# round 6: the headline and every config on the final kernels — smoke, bench.py (defaults), its kernel trace and
# HBM traffic passes, and tools/bench_configs.py over every BASELINE config (4 batches in flight)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh smoke bench prof pmc 'configs:--inflight+4' || exit $?
