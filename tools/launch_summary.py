#!/usr/bin/env python3
"""Per-launch summary of one kernel from a rocprofv3 kernel trace (run_kernel_trace.csv).

    python tools/launch_summary.py TRACE.csv --kernel sq6_scan [--bytes 5.92e9] [--out summary.json]

Reports every launch of the kernel (count, mean, min, max duration) and the launches that overlap no
other launch of ANY kernel on the device (isolated: their duration is the kernel's own time, not a share
of HBM with a neighbour), with the achieved rate of `--bytes` algorithmic bytes per launch against the
8 TB/s spec.  bench.py's roofline `frac` is priced on the isolated (one-in-flight) launches, so this is
the figure the committed profile must reproduce.
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", required=True, help="substring of the kernel name")
    ap.add_argument("--bytes", type=float, default=0.0, help="algorithmic bytes per launch")
    ap.add_argument("--peak", type=float, default=8.0e12)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    mine = [i for i, (_, _, n) in enumerate(rows) if a.kernel in n]
    if not mine:
        raise SystemExit(f"no launch of {a.kernel}")

    def overlaps(i):
        s, e, _ = rows[i]
        for j, (s2, e2, _) in enumerate(rows):
            if j != i and s2 < e and e2 > s:
                return True
        return False

    dur = [(rows[i][1] - rows[i][0]) / 1e6 for i in mine]
    iso = [(rows[i][1] - rows[i][0]) / 1e6 for i in mine if not overlaps(i)]
    out = {"kernel": rows[mine[0]][2], "launches": len(dur), "mean_ms": statistics.mean(dur), "min_ms": min(dur),
           "max_ms": max(dur), "isolated_launches": len(iso)}
    if iso:
        out.update(isolated_mean_ms=statistics.mean(iso), isolated_min_ms=min(iso),
                   isolated_median_ms=statistics.median(iso))
        if a.bytes:
            out["bytes_per_launch"] = a.bytes
            out["isolated_GBps"] = a.bytes / (out["isolated_mean_ms"] * 1e-3) / 1e9
            out["isolated_frac_of_peak"] = out["isolated_GBps"] * 1e9 / a.peak
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
