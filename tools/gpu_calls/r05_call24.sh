set -u
cd $GRAFT_REPO_ROOT
steps=("test:scan_profile")
for rep in 1 2 3; do
  for t in 0 3072; do
    steps+=("cmd:200:tab_${t}_$rep.log:python -u bench.py --tiles $t --steps 400 --warmup 20 --no-cpu-baseline")
  done
done
bash tools/gpu_run.sh "${steps[@]}"
