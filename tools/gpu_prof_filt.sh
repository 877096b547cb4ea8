set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_filt -o run -- python -u tools/bench_configs.py --only C3,C5f > $OUT/prof_filt.log 2>&1 || exit $?
tail -1 $OUT/smoke.log; grep -i "sq8_scan" $OUT/prof_filt/run_kernel_stats.csv | cut -c1-160
