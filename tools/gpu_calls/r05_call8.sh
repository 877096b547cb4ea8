set -u
cd $GRAFT_REPO_ROOT
V="default: sq6_rebound_prefetch=0 sq6_rebound_wgs=1 sq6_rebound_wgs=2 sq6_rebound_prefetch=0,sq6_rebound_wgs=2 sq6_rebound_stride=0"
steps=()
i=0
for v in $V; do
  t=${v#default:}
  steps+=("cmd:150:rb_$i.log:OSK_TESTING_LIB=0 TUNE=$t rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rb_$i -o run -- python -u tools/rebound_diag.py 48")
  i=$((i+1))
done
steps+=("test:sq6")
steps+=("bench:--steps+300+--warmup+20+--no-cpu-baseline")
steps+=("cmd:300:prof_f1.log:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_f1 -o run -- python bench.py --steps 200 --warmup 10 --inflight 1 --no-cpu-baseline")
steps+=("cmd:150:rb_abl.log:OSK_TESTING_LIB=1 TUNE=sq8_mfma_ablate=256 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rb_abl -o run -- python -u tools/rebound_diag.py 48")
bash tools/gpu_run.sh "${steps[@]}"
