set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() { local secs=$1 log=$2; shift 2; echo "== $(date +%T) $*" | tee -a $OUT/steps.log; timeout -k 10 $secs "$@" > $log 2>&1; local rc=$?; echo "   rc=$rc" | tee -a $OUT/steps.log; tail -2 $log | cut -c1-300; case $rc in 0) return 0;; *) exit $rc;; esac; }
run 600 $OUT/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 600 $OUT/filt.jsonl python -u tools/bench_configs.py --only C3,C5f
cat $OUT/filt.jsonl
run 600 $OUT/bench_default.log python bench.py
