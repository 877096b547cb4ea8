set -u
# the driver's default bench line (N=1, b1, CPU baseline), its rocprof kernel stats, b8 / 1.25M lines
export TMPDIR=/tmp
OUT=gpurun_out
run() { local secs=$1 log=$2; shift 2; echo "== $(date +%T) $*" | tee -a $OUT/steps.log; timeout -k 10 $secs "$@" > $log 2>&1; local rc=$?; echo "   rc=$rc" | tee -a $OUT/steps.log; tail -1 $log | cut -c1-200; case $rc in 0) return 0;; *) exit $rc;; esac; }
run 600 $OUT/bench_default.log python bench.py
run 300 $OUT/rocprof.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline
run 300 $OUT/bench_b8.log python bench.py --steps 50 --warmup 3 --batch 8 --no-cpu-baseline
run 300 $OUT/bench_b16.log python bench.py --steps 50 --warmup 3 --batch 16 --no-cpu-baseline
run 300 $OUT/small.log python bench.py --steps 400 --warmup 20 --no-cpu-baseline --rows-per-shard 156250
