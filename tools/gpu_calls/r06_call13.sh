# round 6: the pilot bounds one row per lane (its best approximate score) — the whole GPU suite, then the batched
# configs (C2 b256, C3 b256, C4 b1024)
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh test \
  'cmd:600:cfg13_batched.jsonl:python -u tools/bench_configs.py --only C2,C3,C4 --c2-batches 256 --c3-batches 256 --c4-batches 1024 --steps 6'
