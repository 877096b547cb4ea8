# round 6: the rows kernel's launch-set parameters — first-pass share, pilot rows, quarter size — at C4 b1024 and
# C2 b256 (one process per config; the library's defaults are phase 8, pilot 128 rows, quarters auto)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/tune14.jsonl
: > $OUT
run() {  # run <label> <bench_configs args...>
  local lab=$1; shift
  echo "== $lab" >> $OUT
  timeout -k 10 240 python -u tools/bench_configs.py "$@" >> $OUT 2> gpurun_out/tune14_err.log || { echo "failed: $lab"; exit 1; }
}
C4="--only C4 --c4-batches 1024 --steps 4"
C2="--only C2 --c2-batches 256 --steps 10"
run c4_default $C4
run c4_phase16 $C4 --tune sq8_wide_phase=16
run c4_phase4 $C4 --tune sq8_wide_phase=4
run c4_pilot256 $C4 --tune sq8_wide_pilot_rows=256
run c4_pilot64 $C4 --tune sq8_wide_pilot_rows=64
run c4_q8192 $C4 --tune sq8_wide_quarter_rows=8192
run c4_q32768 $C4 --tune sq8_wide_quarter_rows=32768
run c2_default $C2
run c2_pilot64 $C2 --tune sq8_wide_pilot_rows=64
run c2_pilot256 $C2 --tune sq8_wide_pilot_rows=256
run c2_phase4 $C2 --tune sq8_wide_phase=4
run c2_q4096 $C2 --tune sq8_wide_quarter_rows=4096
run c2_q1024 $C2 --tune sq8_wide_quarter_rows=1024
echo tune-done
# the rows kernel's clocks (testing build), C2 and C4, full / no slow path / streaming only
ABLATE=0,4,1 timeout -k 10 300 python -u tools/wide_ablate.py C2 256 > gpurun_out/clk_c2.log 2>&1 || exit 1
ABLATE=0,4,1 timeout -k 10 300 python -u tools/wide_ablate.py C4 256 > gpurun_out/clk_c4.log 2>&1 || exit 1
echo clocks-done
