# round 6, first call: the whole GPU suite (new: C1 1k queries, C2 b1, C4 MIP at 100M, C5 10 %, whole-batch
# checks, the glds16_run destination probe, the lazy wide copy, rank-local refusals), smoke, default bench
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh test smoke bench:--steps+200
