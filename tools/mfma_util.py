#!/usr/bin/env python3
"""MFMA utilisation from rocprofv3 --pmc counter CSVs (SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_*,
GRBM_GUI_ACTIVE, SQ_INSTS_VALU / SALU / LDS / VMEM_RD) of the MFMA kernels, per kernel over its launches.

  python tools/mfma_util.py OUT.json CSV [CSV ...]

Normalisation (checked against the kernels' own arithmetic): SQ_VALU_MFMA_BUSY_CYCLES sums
busy cycles over all 1,024 SIMDs (256 CUs × 4), GRBM_GUI_ACTIVE sums the launch's cycles over the 8 XCDs,
one MOP = 512 ops (int8: a 16×16×64 MFMA is 128 MOPs and 16 busy SIMD-cycles).  So
  mfma_busy_frac = MFMA_BUSY / (1024 × GRBM_GUI_ACTIVE / 8)   (fraction of SIMD-cycles the matrix core runs)
The launches of one kernel are split into pilot-sized and main-sized by GRBM_GUI_ACTIVE; main-sized ones are
averaged (the int8 path's pilot scores 16 rows per wave)."""
import collections
import csv
import json
import sys

SIMDS, XCDS = 1024, 8


def main():
    out, paths = sys.argv[1], sys.argv[2:]
    per = collections.defaultdict(dict)   # (file, dispatch) -> counters
    names = {}
    for pth in paths:
        for r in csv.DictReader(open(pth)):
            k = r["Kernel_Name"]
            if "mfma" not in k:
                continue
            key = (pth, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] = float(r["Counter_Value"])
            names[key] = k.split("(")[0]
    by_kernel = collections.defaultdict(list)
    for key, c in per.items():
        by_kernel[names[key]].append(c)
    res = {}
    for k, ls in by_kernel.items():
        g = [c.get("GRBM_GUI_ACTIVE", 0.0) for c in ls]
        big = max(g)
        main_ls = [c for c in ls if c.get("GRBM_GUI_ACTIVE", 0.0) >= 0.5 * big]
        avg = {n: sum(c.get(n, 0.0) for c in main_ls) / len(main_ls) for n in main_ls[0]}
        cyc = avg.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        rec = {"launches": len(main_ls), "kernel_cycles": cyc}
        if cyc:
            rec["mfma_busy_frac"] = avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (SIMDS * cyc)
        mops = sum(v for n, v in avg.items() if n.startswith("SQ_INSTS_VALU_MFMA_MOPS"))
        rec["mfma_ops"] = mops * 512
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
            if n in avg:
                rec[n] = avg[n]
        res[k] = rec
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(k, json.dumps(v))


if __name__ == "__main__":
    main()
