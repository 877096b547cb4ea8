set -u
cd $GRAFT_REPO_ROOT
steps=()
for rep in 1 2; do
  for t in 3072 2560 3840; do
    steps+=("cmd:200:tab2_${t}_$rep.log:python -u bench.py --tiles $t --steps 400 --warmup 20 --no-cpu-baseline")
  done
done
bash tools/gpu_run.sh "${steps[@]}"
