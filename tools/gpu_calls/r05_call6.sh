set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "test:wide or sq6 or at_size or full_size" \
  "cmd:240:rebound_diag.log:for sd in 0 1; do TUNE=sq6_rebound_stride=\$sd python -u tools/rebound_diag.py 64 || exit 1; done" \
  "cmd:400:wide_defer.log:for c in C4 C3; do for d in 1 0; do TUNE=sq8_wide_defer=\$d ABLATE=0 python -u tools/wide_ablate.py \$c 256 || exit 1; done; done" \
  "configs:--only+C2,C3,C4+--c2-batches+256+--c3-batches+256+--c4-batches+1024" \
  "bench:--steps+300+--warmup+20+--no-cpu-baseline"
