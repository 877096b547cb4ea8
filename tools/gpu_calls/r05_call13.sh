set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "test:sq6 or comm or profile or bench or at_size" \
  "bench:--steps+500+--warmup+20+--no-cpu-baseline" \
  "cmd:300:bench_f1.log:python -u bench.py --steps 300 --warmup 10 --inflight 1 --no-cpu-baseline" \
  "cmd:300:bench_share.log:python -u bench.py --rank-share 0/8 --steps 3000 --warmup 20 --no-cpu-baseline" \
  "cmd:300:prof_f1.log:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f1 -o run -- python bench.py --steps 200 --warmup 10 --inflight 1 --no-cpu-baseline" \
  "cmd:150:rt_1.log:OSK_TESTING_LIB=0 TUNE=sq6_rebound_retest=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rt_1 -o run -- python -u tools/rebound_diag.py 64" \
  "cmd:150:rt_0.log:OSK_TESTING_LIB=0 TUNE=sq6_rebound_retest=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rt_0 -o run -- python -u tools/rebound_diag.py 64"
