#!/usr/bin/env python3
"""Per launch set of the wide int8 prefilter (pilot, first pass, second pass per 256 queries): duration from the
kernel trace, HBM read/write from the FETCH_SIZE / WRITE_SIZE passes, of one tools/prof_wide.sh directory.

    python tools/wide_launch_sets.py gpurun_out/r05_c4 OUT.json "label" "algorithmic note"

The three runs (trace, FETCH, WRITE) issue the same launches in the same order, so the k-th sq8_wide dispatch is
the same launch in each.  Launches come in sets of three per 256 queries (pilot, first pass, second pass), in
dispatch order; the first set of the run (one-time builds around it) is skipped.  Read bytes = 2 × FETCH_SIZE ×
1024 (gfx950 reports half the bytes of wide coalesced reads; the LDS-DMA ring loads 16 B per lane — the same
correction as tools/pmc_traffic.py's scan kernels; round 4's `profiles/r04b/wide_launch_sets.json` used it too),
write bytes = WRITE_SIZE × 1024."""
import csv
import json
import sys


def dispatches(path, value=None):
    out = []
    for r in csv.DictReader(open(path)):
        if "sq8_wide<" not in r["Kernel_Name"] and "sq8_wide_rows<" not in r["Kernel_Name"]:
            continue
        if value:
            if r["Counter_Name"] != value:
                continue
            out.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        else:
            out.append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
    out.sort()
    return [v for _, v in out]


def main():
    d, out_path, label = sys.argv[1], sys.argv[2], sys.argv[3]
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    ms = dispatches(f"{d}/trace/run_kernel_trace.csv")
    fetch = dispatches(f"{d}/pmc_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = dispatches(f"{d}/pmc_write/run_counter_collection.csv", "WRITE_SIZE")
    n = min(len(ms), len(fetch), len(write)) // 3 * 3
    roles = ["pilot", "first_pass", "second_pass"]
    acc = {r: {"ms": [], "read_GB": [], "write_GB": []} for r in roles}
    for i in range(3, n):   # (the first set skipped)
        r = roles[i % 3]
        acc[r]["ms"].append(ms[i])
        acc[r]["read_GB"].append(2 * fetch[i] * 1024 / 1e9)
        acc[r]["write_GB"].append(write[i] * 1024 / 1e9)
    res = {"label": label, "launch_sets_averaged": (n - 3) // 3, "note": note, "per_256_query_launch_set": {}}
    tot_ms = 0.0
    for r in roles:
        a = acc[r]
        if not a["ms"]:
            continue
        m = sum(a["ms"]) / len(a["ms"])
        rd = sum(a["read_GB"]) / len(a["read_GB"])
        wr = sum(a["write_GB"]) / len(a["write_GB"])
        tot_ms += m
        res["per_256_query_launch_set"][r] = {"ms": round(m, 4), "hbm_read_GB": round(rd, 4),
                                              "hbm_write_GB": round(wr, 4), "read_GBps": round(rd / m * 1e3, 1)}
    res["sq8_wide_ms_per_256"] = round(tot_ms, 4)
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
