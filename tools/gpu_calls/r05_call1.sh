set -u
cd $GRAFT_REPO_ROOT
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
bash tools/gpu_run.sh "test:wide or full_size" \
  "cmd:400:pmc_wide_c4.log:bash tools/pmc_wide_sq.sh C4 256" \
  "cmd:300:pmc_wide_c2.log:bash tools/pmc_wide_sq.sh C2 256" \
  "bench:--rows-per-shard+156250+--steps+2000+--warmup+20+--no-cpu-baseline" \
  "cmd:300:prof_1p25M.log:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_1p25M -o run -- python bench.py --rows-per-shard 156250 --steps 500 --warmup 10 --no-cpu-baseline"
