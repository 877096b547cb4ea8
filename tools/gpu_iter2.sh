set -u
# GPU iteration: parity tests, b1 10M / b1 1.25M benches, rocprof of the latency-kernel micro-benchmark
export TMPDIR=/tmp
OUT=gpurun_out
run() { local secs=$1 log=$2; shift 2; echo "== $(date +%T) $*" | tee -a $OUT/steps.log; timeout -k 10 $secs "$@" > $log 2>&1; local rc=$?; echo "   rc=$rc" | tee -a $OUT/steps.log; tail -3 $log; case $rc in 0) return 0;; *) exit $rc;; esac; }
run 600 $OUT/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 $OUT/bench.log python bench.py --steps 100 --warmup 5 --no-cpu-baseline
run 300 $OUT/small.log python bench.py --steps 400 --warmup 20 --no-cpu-baseline --rows-per-shard 156250
run 300 $OUT/rocprof_small.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_small -o run -- python tools/small_kernels.py
