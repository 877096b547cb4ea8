set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "test:wide or at_size or full_size or prefilter" \
  "cmd:400:wide_cnt2.log:ABLATE=0 python -u tools/wide_ablate.py C4 256 && ABLATE=0 python -u tools/wide_ablate.py C3 256" \
  "configs:--only+C2,C3,C4+--c2-batches+256+--c3-batches+256+--c4-batches+1024"
