set -u
export TMPDIR=/tmp
OUT=gpurun_out
run() { local secs=$1 log=$2; shift 2; echo "== $(date +%T) $*" | tee -a $OUT/steps.log; timeout -k 10 $secs "$@" > $log 2>&1; local rc=$?; echo "   rc=$rc" | tee -a $OUT/steps.log; tail -2 $log | cut -c1-300; case $rc in 0) return 0;; *) exit $rc;; esac; }
run 900 $OUT/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
bash tools/gpu_ab.sh "--batch 16" "--batch 32" "--batch 32 --tune sq8_mfma_queries=16" "--batch 64" "--batch 64 --tune sq8_mfma_queries=16" "--batch 96 --mfma-min-batch 100000" "--batch 128 --mfma-min-batch 100000" "--batch 128" "--batch 256"
