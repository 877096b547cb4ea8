set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "test:sq6 or concurrency or lifecycle" \
  "cmd:300:bench_share.log:python -u bench.py --rank-share 0/8 --steps 3000 --warmup 20 --no-cpu-baseline" \
  "cmd:300:prof_share.log:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_share -o run -- python bench.py --rank-share 0/8 --steps 500 --warmup 10 --inflight 1 --no-cpu-baseline" \
  "bench:--steps+200+--warmup+10+--no-cpu-baseline"
