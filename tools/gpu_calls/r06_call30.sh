# round 6: the 6-bit pass at the N = 8 share (1.25M rows) against its tiling — resident slots per CU, rows per
# tile (bench.py --rank-share 0/8, 4 in flight)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tune30.jsonl
: > $OUT
run() {
  local lab=$1; shift
  echo "== $lab" >> $OUT
  timeout -k 10 240 python -u bench.py --rank-share 0/8 --steps 300 --warmup 20 --no-cpu-baseline "$@" > gpurun_out/tune30_one.log 2>&1 || { echo "failed: $lab"; tail -5 gpurun_out/tune30_one.log; exit 1; }
  grep '^{' gpurun_out/tune30_one.log | tail -1 >> $OUT
}
run default
run slots2 --tune tile_slots_per_cu=2
run slots8 --tune tile_slots_per_cu=8
run minrows512 --tune tile_min_rows=512
run minrows2048 --tune tile_min_rows=2048
run default_b
echo tune-done
