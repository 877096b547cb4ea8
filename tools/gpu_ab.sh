set -u
# A/B of bench variants: each arg is one quoted set of bench flags
export TMPDIR=/tmp
OUT=gpurun_out
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline $args > $OUT/ab_$i.log 2>&1 || { echo "rc=$? for $args"; tail -5 $OUT/ab_$i.log; exit 1; }
  tail -1 $OUT/ab_$i.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$args |', round(d['value']), 'QPS scan_ms', round(r['scan_ms_avg'],3), 'step_ms', round(d['ms_per_step'],3))"
done
