# final tree (after the cold parameters in LDS): every GPU test, smoke, default bench, rocprof stats of it,
# and the batched configs
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.log
bash tools/gpu_run.sh smoke bench prof "configs:--only+C2,C3,C4+--c2-batches+256+--c3-batches+1,256+--c4-batches+1024+--steps+20"
