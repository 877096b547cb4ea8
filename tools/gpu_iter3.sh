set -u
# int8 MFMA prefilter: parity tests, then batch sweep (prefilter MFMA vs bf16x3 MFMA path)
export TMPDIR=/tmp
OUT=gpurun_out
run() { local secs=$1 log=$2; shift 2; echo "== $(date +%T) $*" | tee -a $OUT/steps.log; timeout -k 10 $secs "$@" > $log 2>&1; local rc=$?; echo "   rc=$rc" | tee -a $OUT/steps.log; tail -3 $log | cut -c1-600; case $rc in 0) return 0;; *) exit $rc;; esac; }
run 600 $OUT/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for b in 2 8 16 32 64; do
  run 300 $OUT/b$b.log python bench.py --steps 20 --warmup 2 --no-cpu-baseline --batch $b --mfma-min-batch 100000
done
run 300 $OUT/b8_valu.log python bench.py --steps 20 --warmup 2 --no-cpu-baseline --batch 8 --sq8-mfma-min 0
