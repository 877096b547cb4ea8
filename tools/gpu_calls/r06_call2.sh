# round 6: the barrier-free wide kernel (sq8_wide_rows, ≤ 128 dims) — its parity tests, then C2 b256 / C4 b1024
# with it (default) and without it (sq8_wide_rows=0), one batch in flight
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh test:test_gpu_wide \
  'cmd:600:cfg_rows1.jsonl:python -u tools/bench_configs.py --only C2,C4 --c4-batches 1024 --c2-batches 256 --steps 8' \
  'cmd:600:cfg_rows0.jsonl:python -u tools/bench_configs.py --only C2,C4 --c4-batches 1024 --c2-batches 256 --steps 8 --tune sq8_wide_rows=0'
