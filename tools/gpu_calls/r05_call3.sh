set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh "test" \
  "cmd:300:wide_c4.log:ABLATE=0,1,64 python -u tools/wide_ablate.py C4 256" \
  "cmd:300:wide_c2.log:ABLATE=0 python -u tools/wide_ablate.py C2 256" \
  "cmd:300:wide_c3.log:ABLATE=0,1,64 python -u tools/wide_ablate.py C3 256" \
  "configs:--only+C2,C3,C4+--c2-batches+256+--c3-batches+256+--c4-batches+1024"
