set -u
# HBM traffic of the headline bench (C3, b1, prefilter path): two rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE: they cannot share a pass), then tools/pmc_traffic.py applies the gfx950
# x2 FETCH correction for the 16-B-per-lane streaming scans (MI355X_MICROARCH.md, HBM section).
export TMPDIR=/tmp
OUT=gpurun_out
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 || exit $?
python tools/pmc_traffic.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv --out $OUT/pmc_traffic_c3_b1.json > $OUT/pmc_summary.txt 2>&1
