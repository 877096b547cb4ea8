"""Summarise a gpu_iter.sh run (bench lines + rocprof kernel stats)."""
import csv, json, os, sys
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in ("bench", "bench_b8", "small"):
    p = os.path.join(out, f + ".log")
    if not os.path.exists(p):
        continue
    for line in open(p):
        if line.startswith("{"):
            d = json.loads(line)
            print(f"{f:9s} B={d['config']['batch']} rows={d['config']['rows']} QPS={d['value']:.1f} "
                  f"ms/step={d['ms_per_step']:.4f} gpu_ms/step={d['gpu_event_ms_per_step']:.4f} "
                  f"scan_ms={d['roofline']['scan_ms_avg']:.4f} frac={d['roofline']['frac']:.3f} "
                  f"{d.get('prefilter')}")
p = os.path.join(out, "prof", "run_kernel_stats.csv")
if os.path.exists(p):
    for r in csv.DictReader(open(p)):
        print(f"  {r['Name'][:60]:60s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:10.1f} us")
