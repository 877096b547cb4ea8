set -u
# kernel breakdown of the int8 MFMA prefilter at C3 b16 (pilot, pilot merge, main scan, settle)
export TMPDIR=/tmp
OUT=gpurun_out
run() { local secs=$1 log=$2; shift 2; echo "== $(date +%T) $*" | tee -a $OUT/steps.log; timeout -k 10 $secs "$@" > $log 2>&1; local rc=$?; echo "   rc=$rc" | tee -a $OUT/steps.log; tail -2 $log | cut -c1-300; case $rc in 0) return 0;; *) exit $rc;; esac; }
run 600 $OUT/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 $OUT/rocprof_b16.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_b16 -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline --batch 16
