# round 6: C4 b1024 on the rows kernel against its pilot rows (the first pass's floors) and first-pass share
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tune31.jsonl
: > $OUT
run() {
  local lab=$1; shift
  echo "== $lab" >> $OUT
  timeout -k 10 240 python -u tools/bench_configs.py --only C4 --c4-batches 1024 --steps 4 "$@" >> $OUT 2> gpurun_out/tune31_err.log || { echo "failed: $lab"; exit 1; }
}
run default
run pilot256 --tune sq8_wide_pilot_rows=256
run pilot512 --tune sq8_wide_pilot_rows=512
run phase4 --tune sq8_wide_phase=4
run pilot256_phase4 --tune sq8_wide_pilot_rows=256 --tune sq8_wide_phase=4
run default_b
echo tune-done
