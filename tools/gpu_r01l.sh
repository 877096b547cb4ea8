set -u
# round-1 closing run: GPU parity tests, smoke, default bench line + rocprof stats, every config, b32 prefilter
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() { local secs=$1 log=$2; shift 2; echo "== $(date +%T) $*" | tee -a $OUT/steps.log; timeout -k 10 $secs "$@" > $log 2>&1; local rc=$?; echo "   rc=$rc" | tee -a $OUT/steps.log; tail -1 $log | cut -c1-300; case $rc in 0) return 0;; *) exit $rc;; esac; }
run 600 $OUT/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run 200 $OUT/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 600 $OUT/bench_default.log python bench.py
run 300 $OUT/rocprof.log rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline
run 900 $OUT/configs_sweep.jsonl python -u tools/bench_configs.py --c4-batches 1,32,1024
export ABLATE=0
run 200 $OUT/b32_c4.log python -u tools/mfma_ablate.py C4 32
run 200 $OUT/b32_c3.log python -u tools/mfma_ablate.py C3 32
