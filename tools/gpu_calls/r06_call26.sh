# round 6, final tree: the whole GPU suite, smoke, then C3 / C4 b32 on the library's defaults
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh test smoke \
  'cmd:400:cfg26_b32.jsonl:python -u tools/bench_configs.py --only C3,C4 --c3-batches 32 --c4-batches 32 --steps 8 --inflight 4' || exit $?
