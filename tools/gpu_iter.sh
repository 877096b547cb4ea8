set -u
# quick GPU iteration: parity tests, b1/b8 bench lines without the CPU baseline, a 1.25M-row bench
# (the per-GPU size at N=8), rocprof stats of the b1 bench
export TMPDIR=/tmp
OUT=gpurun_out
run() { local secs=$1 log=$2; shift 2; echo "== $(date +%T) $*" | tee -a $OUT/steps.log; timeout -k 10 $secs "$@" > $log 2>&1; local rc=$?; echo "   rc=$rc" | tee -a $OUT/steps.log; tail -3 $log; case $rc in 0) return 0;; *) exit $rc;; esac; }
run 600 $OUT/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run 300 $OUT/bench.log python bench.py --steps 100 --warmup 5 --no-cpu-baseline
run 300 $OUT/bench_b8.log python bench.py --steps 50 --warmup 3 --batch 8 --no-cpu-baseline
run 300 $OUT/small.log python bench.py --steps 400 --warmup 20 --no-cpu-baseline --rows-per-shard 156250
run 300 $OUT/rocprof.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline
