#!/usr/bin/env bash
# GPU-box check run (used through gpurun): parity tests, smoke, a short bench and a rocprofv3
# kernel-trace summary.  Each GPU step has its own time limit; a crash/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-all}
run() {  # run <seconds> <logfile> cmd...
  local secs=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "   rc=$rc ($(tail -c 300 "$log" | tr '\n' ' ' | cut -c1-300))" | tee -a "$OUT/steps.log"
  case $rc in 124|134|137|139) echo "fatal rc=$rc, stopping"; exit $rc;; esac
  return 0
}
rocm-smi --showproductname > "$OUT/rocm_smi.txt" 2>&1 || true
if [[ $STEPS == all || $STEPS == *test* ]]; then
  run 900 "$OUT/pytest_gpu.log" python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  run 300 "$OUT/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  run 600 "$OUT/bench.log" python bench.py --steps ${BENCH_STEPS:-100} --warmup 5
  grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  run 600 "$OUT/rocprof.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python bench.py --steps 30 --warmup 3 --no-cpu-baseline
fi
echo done
