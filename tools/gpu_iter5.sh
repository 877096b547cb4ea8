set -u
export TMPDIR=/tmp
OUT=gpurun_out
run() { local secs=$1 log=$2; shift 2; echo "== $(date +%T) $*" | tee -a $OUT/steps.log; timeout -k 10 $secs "$@" > $log 2>&1; local rc=$?; echo "   rc=$rc" | tee -a $OUT/steps.log; tail -2 $log | cut -c1-300; case $rc in 0) return 0;; *) exit $rc;; esac; }
run 600 $OUT/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 200 $OUT/ablate.log python tools/mfma_ablate.py
bash tools/gpu_ab.sh "--batch 1" "--batch 8" "--batch 16" "--batch 64" "--batch 1 --rows-per-shard 156250 --steps 200"
