set -u
cd $GRAFT_REPO_ROOT
steps=("test:rebound_schedules or test_many_tiles")
i=0
for r in 1 0 1 0; do
  steps+=("cmd:150:rt_$i.log:OSK_TESTING_LIB=0 TUNE=sq6_rebound_retest=$r rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rt_$i -o run -- python -u tools/rebound_diag.py 64")
  i=$((i+1))
done
steps+=("cmd:600:pmc_wide.log:bash tools/pmc_wide_sq.sh C4 256")
bash tools/gpu_run.sh "${steps[@]}"
