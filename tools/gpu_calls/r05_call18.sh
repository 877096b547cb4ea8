set -u
cd $GRAFT_REPO_ROOT
steps=()
for t in 0 3072 2048 1024 1536; do
  steps+=("cmd:200:tiles_f1_$t.log:python -u bench.py --tiles $t --steps 300 --warmup 10 --inflight 1 --no-cpu-baseline")
  steps+=("cmd:200:tiles_f4_$t.log:python -u bench.py --tiles $t --steps 300 --warmup 10 --no-cpu-baseline")
done
bash tools/gpu_run.sh "${steps[@]}"
