set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "test:sq6 or full_size or at_size or large_view or filter" \
  "bench:--steps+400+--warmup+20+--no-cpu-baseline" \
  "cmd:300:bench_f1.log:python -u bench.py --steps 300 --warmup 10 --inflight 1 --no-cpu-baseline" \
  "configs:--only+C3,C4,C5i,C5f+--c3-batches+1,32+--c4-batches+1,32+--c5f-modes+1:0+--inflight+4"
