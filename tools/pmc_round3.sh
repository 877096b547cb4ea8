set -e
export TMPDIR=/tmp
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
C2="python tools/bench_configs.py --only C2 --c2-batches 256 --steps 5"
C4="python tools/bench_configs.py --only C4 --c4-batches 32 --steps 5"
for name in c3b1:B c2b256:C2 c4b32:C4; do
  n=${name%%:*}; v=${name#*:}; cmd=${!v}
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${n}_fetch -o run -- $cmd > gpurun_out/pmc_${n}_fetch.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${n}_write -o run -- $cmd > gpurun_out/pmc_${n}_write.log 2>&1
  python tools/pmc_traffic.py gpurun_out/pmc_${n}_fetch/run_counter_collection.csv gpurun_out/pmc_${n}_write/run_counter_collection.csv --out gpurun_out/pmc_${n}.json > gpurun_out/pmc_${n}.txt 2>&1
done
