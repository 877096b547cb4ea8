set -u
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh \
  "cmd:900:tls_24.log:python -u tools/bench_configs.py --only C3,C4,C5i,C5f --c3-batches 1,32 --c4-batches 1,32 --c5f-modes 1:0 --inflight 4 --tune tile_large_slots=24" \
  "cmd:900:tls_12.log:python -u tools/bench_configs.py --only C3,C4,C5i,C5f --c3-batches 1,32 --c4-batches 1,32 --c5f-modes 1:0 --inflight 4 --tune tile_large_slots=12"
