# round 6: C3 b256 (ring kernel) against its pilot size and first-pass share, now that the pilot bounds one row
# per lane (the insertions cost 1.1 of 3.9 ms: profiles/r06/wide_ablate_c3_b256_ring.log)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tune28.jsonl
: > $OUT
run() {
  local lab=$1; shift
  echo "== $lab" >> $OUT
  timeout -k 10 240 python -u tools/bench_configs.py --only C3 --c3-batches 256 --steps 6 "$@" >> $OUT 2> gpurun_out/tune28_err.log || { echo "failed: $lab"; exit 1; }
}
run default
run pilot512 --tune sq8_wide_pilot_rows=512
run pilot1024 --tune sq8_wide_pilot_rows=1024
run phase4 --tune sq8_wide_phase=4
run phase16 --tune sq8_wide_phase=16
run default_b
echo tune-done
