set -u
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --rows-per-shard 156250 > gpurun_out/small.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_small -o run -- python bench.py --steps 100 --warmup 5 --no-cpu-baseline --rows-per-shard 156250 > gpurun_out/small_prof.log 2>&1
