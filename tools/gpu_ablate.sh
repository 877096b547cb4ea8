set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
for a in "C4 32" "C3 32"; do
  timeout -k 10 300 python -u tools/mfma_ablate.py $a >> $OUT/ablate.log 2>&1 || exit $?
done
cat $OUT/ablate.log
