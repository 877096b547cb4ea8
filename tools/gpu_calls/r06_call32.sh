# round 6, final tree: every BASELINE config with 4 batches in flight, plus C3 / C4 b32
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'configs:--inflight+4' \
  'cmd:400:cfg32_b32.jsonl:python -u tools/bench_configs.py --only C3,C4 --c3-batches 32 --c4-batches 32 --steps 10 --inflight 4' || exit $?
