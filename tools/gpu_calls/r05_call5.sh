set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "test:sq6 or full_size or concurrency" \
  "bench:--steps+500+--warmup+20+--no-cpu-baseline" \
  "cmd:300:bench_f1.log:python -u bench.py --steps 300 --warmup 10 --inflight 1 --no-cpu-baseline" \
  "cmd:300:bench_share.log:python -u bench.py --rank-share 0/8 --steps 3000 --warmup 20 --no-cpu-baseline" \
  "cmd:300:prof_f1.log:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f1 -o run -- python bench.py --steps 200 --warmup 10 --inflight 1 --no-cpu-baseline" \
  "cmd:600:wide_phase.log:for ph in 0 4 8 16; do TUNE=sq8_wide_phase=\$ph ABLATE=0 python -u tools/wide_ablate.py C4 256 || exit 1; done; for pr in 256 512; do TUNE=sq8_wide_pilot_rows=\$pr ABLATE=0 python -u tools/wide_ablate.py C4 256 || exit 1; done"
