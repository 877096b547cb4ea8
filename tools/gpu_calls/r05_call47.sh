# final-tree evidence (round 5, after the one-statement DMAs): every GPU test, smoke, the default bench,
# rocprof stats, FETCH/WRITE PMC of the bench, one-in-flight bench + trace, and the every-config sweep
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.log
bash tools/gpu_run.sh smoke bench prof pmc \
  "cmd:300:bench_f1.log:python -u bench.py --steps 300 --warmup 10 --inflight 1 --no-cpu-baseline" \
  "cmd:300:prof_f1.log:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f1 -o run -- python bench.py --steps 200 --warmup 10 --inflight 1 --no-cpu-baseline" \
  "configs:--steps+20"
