set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
export ABLATE=0,3
for t in "" "sq8_mfma_nt=0" "sq8_mfma_queries=16" "tile_slots_per_cu=3" "tile_slots_per_cu=8"; do
  for c in "C3 32" "C4 32"; do
    TUNE="$t" timeout -k 10 200 python -u tools/mfma_ablate.py $c 2>&1 | grep -v amdgpu.ids >> $OUT/ablate2.log || exit $?
  done
done
cat $OUT/ablate2.log
