#!/usr/bin/env bash
# One parameterised GPU-box runner (used through gpurun).  Each argument is a step; every step that
# touches the GPU runs under its own time limit, and a crash / abort / timeout ends the script (no
# further GPU step runs after a fault).  Logs land in gpurun_out/.
#
#   tools/gpu_run.sh test                 pytest -m gpu (all GPU parity tests)
#   tools/gpu_run.sh test:K_EXPR          pytest -m gpu -k K_EXPR
#   tools/gpu_run.sh smoke                __graft_entry__.smoke()
#   tools/gpu_run.sh bench[:ARGS]         python bench.py ARGS   (ARGS "+"-separated, e.g. bench:--batch+32)
#   tools/gpu_run.sh prof[:ARGS]          rocprofv3 --kernel-trace --stats of a short bench.py ARGS run
#   tools/gpu_run.sh pmc[:ARGS]           FETCH_SIZE and WRITE_SIZE passes (separate runs) + tools/pmc_traffic.py
#   tools/gpu_run.sh mfmapmc[:ARGS]       SQ_INSTS_VALU_MFMA_MOPS_* / SQ_VALU_MFMA_BUSY_CYCLES pass of bench.py ARGS
#   tools/gpu_run.sh configs[:ARGS]       tools/bench_configs.py ARGS (every BASELINE config)
#   tools/gpu_run.sh rehearse             bench.py at N = 2/4/8 gloo ranks on the one GPU, cross-N parity
#   tools/gpu_run.sh 'cmd:SECS:LOG:CMD'   any other command (CMD run by bash)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"

run() {  # run <seconds> <logfile> cmd...
  local secs=$1 log=$2; shift 2
  echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "   rc=$rc ($(tail -c 300 "$log" | tr '\n' ' ' | cut -c1-300))" | tee -a "$OUT/steps.log"
  if [[ $rc != 0 ]]; then echo "step failed rc=$rc, stopping"; exit $rc; fi
}
args() { echo "${1//+/ }"; }   # step args are "+"-separated (bench:--batch+32)

for step in "$@"; do
  name=${step%%:*}
  rest=""; [[ $step == *:* ]] && rest=${step#*:}
  case $name in
    test)
      if [[ -n $rest ]]; then
        run 900 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
            --timeout-method thread -k "$rest"
      else
        run 1100 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
            --timeout-method thread
      fi ;;
    smoke) run 300 "$OUT/smoke.log" python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 600 "$OUT/bench.log" python -u bench.py $(args "$rest")
           grep '^{' "$OUT/bench.log" > "$OUT/bench.json" || true ;;
    prof)  run 300 "$OUT/rocprof.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
               python bench.py --steps 30 --warmup 3 --no-cpu-baseline $(args "$rest") ;;
    pmc)   run 150 "$OUT/pmc_fetch.log" timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv \
               -d "$OUT/pmc_fetch" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline $(args "$rest")
           run 150 "$OUT/pmc_write.log" timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv \
               -d "$OUT/pmc_write" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline $(args "$rest")
           python tools/pmc_traffic.py "$OUT/pmc_fetch/run_counter_collection.csv" \
               "$OUT/pmc_write/run_counter_collection.csv" --out "$OUT/pmc_traffic.json" > "$OUT/pmc_summary.txt" 2>&1 ;;
    mfmapmc)
           run 150 "$OUT/pmc_mfma.log" timeout -s KILL 140 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 \
               SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
               -d "$OUT/pmc_mfma" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline $(args "$rest") ;;
    configs) run 1000 "$OUT/configs_sweep.jsonl" python -u tools/bench_configs.py $(args "$rest") ;;
    rehearse) run 900 "$OUT/rehearse.log" bash tools/gpu_rehearse.sh ;;
    cmd)   secs=${rest%%:*}; rest=${rest#*:}; log=${rest%%:*}; c=${rest#*:}
           run "$secs" "$OUT/$log" bash -c "$c" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
