set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "test:sq6 or full_size or comm or shard_query or merge" \
  "cmd:150:rb_p.log:OSK_TESTING_LIB=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rb_p -o run -- python -u tools/rebound_diag.py 64" \
  "bench:--steps+500+--warmup+20+--no-cpu-baseline" \
  "cmd:300:bench_f1.log:python -u bench.py --steps 300 --warmup 10 --inflight 1 --no-cpu-baseline" \
  "cmd:300:prof_f1.log:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f1 -o run -- python bench.py --steps 200 --warmup 10 --inflight 1 --no-cpu-baseline"
