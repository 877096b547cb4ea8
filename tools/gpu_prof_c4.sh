set -u
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
export ABLATE=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python -u tools/mfma_ablate.py C4 32 > $OUT/prof_c4.log 2>&1 || exit $?
cut -d, -f1-5 $OUT/prof_c4/run_kernel_stats.csv | head -12
