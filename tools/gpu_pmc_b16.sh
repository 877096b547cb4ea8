set -u
# HBM traffic of the int8 MFMA prefilter (C3 b16): FETCH_SIZE and WRITE_SIZE passes
export TMPDIR=/tmp
OUT=gpurun_out
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc16_fetch -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --batch 16 > $OUT/pmc16_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc16_write -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --batch 16 > $OUT/pmc16_write.log 2>&1 || exit $?
python tools/pmc_traffic.py $OUT/pmc16_fetch/run_counter_collection.csv $OUT/pmc16_write/run_counter_collection.csv --out $OUT/pmc_traffic_c3_b16.json > $OUT/pmc16_summary.txt 2>&1
cat $OUT/pmc16_summary.txt
