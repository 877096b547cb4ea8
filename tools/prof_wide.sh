#!/usr/bin/env bash
# rocprofv3 evidence for the wide int8 prefilter on one BASELINE config (tools/bench_configs.py): a kernel
# trace + stats run, then FETCH_SIZE and WRITE_SIZE passes (separate runs), summarised by tools/pmc_traffic.py.
#   tools/prof_wide.sh NAME "BENCH_CONFIGS_ARGS"     → gpurun_out/NAME/
#   e.g. tools/prof_wide.sh r05_c4 "--only C4 --c4-batches 1024 --steps 3"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04b}
ARGS=${2:-"--only C4 --c4-batches 1024 --steps 3"}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 tools/bench_configs.py $ARGS > "$OUT/trace.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 tools/bench_configs.py $ARGS > "$OUT/pmc_fetch.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 tools/bench_configs.py $ARGS > "$OUT/pmc_write.log" 2>&1 || exit $?
python3 tools/pmc_traffic.py "$OUT/pmc_fetch/run_counter_collection.csv" "$OUT/pmc_write/run_counter_collection.csv" \
    --out "$OUT/pmc_traffic.json" > "$OUT/pmc_summary.txt" 2>&1
echo done
