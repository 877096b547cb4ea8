set -u
# every BASELINE config on one MI355X at HEAD (tools/bench_configs.py), one JSON line per (config, batch)
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u tools/bench_configs.py --c4-batches 1,32,1024 > $OUT/configs_sweep.jsonl 2> $OUT/configs_sweep.err
rc=$?; echo "rc=$rc"; tail -3 $OUT/configs_sweep.err; exit $rc
