#!/usr/bin/env bash
# Batched-path check on the GPU box: its parity tests, then benches at several batch sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
run() {
  local secs=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "   rc=$rc ($(tail -c 400 "$log" | tr '\n' ' ' | cut -c1-400))" | tee -a "$OUT/steps.log"
  case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
  return 0
}
run 600 "$OUT/pytest_batched.log" python -m pytest tests/test_gpu_batched.py -q -x -p no:cacheprovider --timeout 300
run 900 "$OUT/pytest_gpu.log" python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300
for b in ${BATCHES:-16 64 256 1024}; do
  run 600 "$OUT/bench_b$b.log" python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --batch $b --no-cpu-baseline
done
run 600 "$OUT/rocprof_b256.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_b256" -o run -- \
    python bench.py --steps 10 --warmup 2 --batch 256 --no-cpu-baseline
echo done
