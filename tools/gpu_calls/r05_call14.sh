set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh \
  "cmd:700:prof_c3.log:bash tools/prof_wide.sh r05_c3 '--only C3 --c3-batches 256 --steps 3'" \
  "cmd:700:prof_c4.log:bash tools/prof_wide.sh r05_c4 '--only C4 --c4-batches 1024 --steps 3'" \
  "cmd:600:pmc_wide_c3.log:bash tools/pmc_wide_sq.sh C3 256" \
  "configs:--inflight+4"
