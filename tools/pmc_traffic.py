#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch per kernel.

  python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [--out f.json]

Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read (16 B per
lane), so read bytes = 2 × FETCH_SIZE × 1024 for such kernels (the scan kernels); WRITE_SIZE is exact
for 16-B streaming stores.  Reported per kernel: mean over its dispatches.
"""
import argparse
import csv
import json
from collections import defaultdict


def load(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--out")
    a = ap.parse_args()
    f, n = load(a.fetch)
    w, _ = load(a.write)
    out = {}
    for k in f:
        # 16-B-per-lane streaming loads: apply the gfx950 ×2 FETCH correction
        # (sq6_scan mixes 16-B and 8-B loads: its ×2-corrected bytes match the 5.92 GB of 6-bit codes +
        # bound terms per C3 search to 0.2 %, profiles/r03b/; sq8_mfma and mfma_cand stream 16-B LDS-DMA)
        wide = any(t in k for t in ("scan_f32<", "scan_i8<", "sq8_scan<", "sq6_scan<", "sq8_mfma<", "mfma_cand<"))
        rd = f[k] * 1024 * (2 if wide else 1)
        wr = w.get(k, 0.0) * 1024
        out[k] = {"dispatches": n[k], "fetch_kib_raw": f[k], "write_kib_raw": w.get(k),
                  "read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr, "fetch_x2_applied": wide}
        print(f"{k[:70]:70s} n={n[k]:3d} read={rd/1e9:9.4f} GB write={wr/1e9:9.4f} GB")
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
