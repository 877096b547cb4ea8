set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] || exit $rc
export ABLATE=0,3
for c in "C4 32" "C3 32"; do
  timeout -k 10 200 python -u tools/mfma_ablate.py $c 2>&1 | grep -v amdgpu.ids >> $OUT/ablate.log || exit $?
done
cat $OUT/ablate.log
timeout -k 10 600 python -u tools/bench_configs.py --only C4 --c4-batches 32,256,1024 2>&1 | grep -v amdgpu.ids > $OUT/c4.jsonl; rc=$?; cat $OUT/c4.jsonl; exit $rc
