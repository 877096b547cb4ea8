set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "test:wide or at_size or full_size" \
  "cmd:500:wide_sync.log:for c in C4 C3; do for sy in 1 0; do TUNE=sq8_wide_sync=\$sy ABLATE=0 python -u tools/wide_ablate.py \$c 256 || exit 1; done; done" \
  "configs:--only+C2,C3,C4+--c2-batches+256+--c3-batches+256+--c4-batches+1024"
