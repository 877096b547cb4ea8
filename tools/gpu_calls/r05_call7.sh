set -u
cd $GRAFT_REPO_ROOT
V="default: sq6_rebound_prefetch=0 sq6_rebound_prefetch=0,sq6_rebound_wgs=2 sq6_rebound_wgs=1 sq8_mfma_ablate=256 sq8_mfma_ablate=512"
steps=("test:sq6 or shard_query or comm_world")
i=0
for v in $V; do
  t=${v#default:}
  steps+=("cmd:150:rb_$i.log:TUNE=$t rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rb_$i -o run -- python -u tools/rebound_diag.py 48")
  i=$((i+1))
done
steps+=("bench:--steps+300+--warmup+20+--no-cpu-baseline")
steps+=("cmd:300:bench_f1.log:python -u bench.py --steps 300 --warmup 10 --inflight 1 --no-cpu-baseline")
bash tools/gpu_run.sh "${steps[@]}"
