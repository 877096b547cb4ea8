# round 6: NaN keys are never hits (make_key), the barrier-free wide kernel's tests, then C2 b256 / C4 b1024 A/B
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_gpu_nan or test_gpu_wide' \
  'cmd:600:cfg_rows1.jsonl:python -u tools/bench_configs.py --only C2,C4 --c4-batches 1024 --c2-batches 256 --steps 8' \
  'cmd:600:cfg_rows0.jsonl:python -u tools/bench_configs.py --only C2,C4 --c4-batches 1024 --c2-batches 256 --steps 8 --tune sq8_wide_rows=0'
