set -u
# A/B: scan workgroup tiles per view at the N=8 per-GPU size (1.25M rows) and at 10M rows
export TMPDIR=/tmp
OUT=gpurun_out
for t in 512 1024 2048 4096; do
  timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --rows-per-shard 156250 --tiles $t > $OUT/tiles_small_$t.log 2>&1 || exit $?
done
for t in 2048 4096 8192; do
  timeout -k 10 120 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --tiles $t > $OUT/tiles_big_$t.log 2>&1 || exit $?
done
