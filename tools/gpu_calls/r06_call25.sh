# round 6: C4 b32 — the 4-slot ring instances (2 workgroups per CU) with lane-compact insertions against the
# default 2-slot ring (4 per CU, per-query insertions); parity of ring depths; SQ passes of the 4-slot run
set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh 'test:test_mfma_ring_depths or test_prefilter_batches_and_k' \
  'cmd:300:cfg25_ring2.jsonl:python -u tools/bench_configs.py --only C4 --c4-batches 32 --steps 8' \
  'cmd:300:cfg25_ring4.jsonl:python -u tools/bench_configs.py --only C4 --c4-batches 32 --steps 8 --tune sq8_mfma_ring=4' \
  'cmd:300:cfg25_ring2b.jsonl:python -u tools/bench_configs.py --only C4 --c4-batches 32 --steps 8' \
  'cmd:300:cfg25_ring4b.jsonl:python -u tools/bench_configs.py --only C4 --c4-batches 32 --steps 8 --tune sq8_mfma_ring=4' || exit $?
