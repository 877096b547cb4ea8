set -u
# A/B: view tiles in whole rounds of both scan kernels' residency (12 = lcm(3, 4) slots per CU) vs default
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
export ABLATE=0
for t in "" "tiles_target=12288" "tiles_target=6144"; do
  for c in "C4 32" "C3 32"; do
    TUNE="$t" timeout -k 10 200 python -u tools/mfma_ablate.py $c 2>&1 | grep -v amdgpu.ids >> $OUT/tiles12.log || exit $?
  done
  tt=""; [ -n "$t" ] && tt="--tune $t"
  echo "== $t" >> $OUT/tiles12.log
  timeout -k 10 300 python -u tools/bench_configs.py --only C3 $tt 2>&1 | grep -v amdgpu.ids >> $OUT/tiles12.log || exit $?
done
cat $OUT/tiles12.log
