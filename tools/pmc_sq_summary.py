#!/usr/bin/env python3
"""Summarise the SQ instruction-mix / MFMA-busy passes of tools/pmc_wide_sq.sh (row n2 of the coverage table).

    python tools/pmc_sq_summary.py OUT.json DIR_PASS1 DIR_PASS2 [label]

Per kernel launch kind (pilot, first pass, second pass: launches told apart by GRBM_GUI_ACTIVE size within a
search), averaged over the searches of the run.  Normalisation (MI355X_MICROARCH.md, rocprofv3 PMC section):
GRBM_GUI_ACTIVE sums the launch's cycles over the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES sums busy cycles over the
1,024 SIMDs; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over waves; one
v_mfma_i32_16x16x64_i8 = 64 MOPS_I8 (16·16·64·2 ops / 512).  So
  mfma_busy   = MFMA_BUSY / (1024 · GRBM / 8)                  (fraction of SIMD-cycles the matrix core runs)
  n_mfma      = MOPS_I8 / 64;  X per MFMA = SQ_INSTS_X / n_mfma
  wave split  = WAIT_ANY (parked: s_waitcnt / barrier), WAIT_INST_ANY (issue-stalled), ACTIVE_INST_ANY (issuing),
                each over SQ_WAVE_CYCLES."""
import collections
import csv
import json
import os
import sys

SIMDS, XCDS, MOPS_PER_MFMA = 1024, 8, 64


def load(d):
    per, names = collections.defaultdict(dict), {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        names[int(r["Dispatch_Id"])] = r["Kernel_Name"].split("(")[0]
    return per, names


def main():
    out, d1, d2 = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    p1, n1 = load(d1)
    p2, _ = load(d2)
    # launches in dispatch order, grouped per search: the wide path issues pilot, first pass, second pass
    ids1, ids2 = sorted(p1), sorted(p2)
    # (KINDS="pilot,main": sq8_mfma's two launches per batch, tools/pmc_mfma_sq.sh)
    kinds = os.environ.get("KINDS", "pilot,first_pass,second_pass").split(",")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for j, (a, b) in enumerate(zip(ids1, ids2)):
        k = kinds[j % len(kinds)]
        c = dict(p1[a])
        c.update({n: v for n, v in p2[b].items() if n != "GRBM_GUI_ACTIVE"})
        for n, v in c.items():
            acc[k][n] += v
        cnt[k] += 1
    res = {"label": label, "kernel": n1[ids1[0]] if ids1 else None}
    for k in kinds:
        if not cnt[k]:
            continue
        c = {n: v / cnt[k] for n, v in acc[k].items()}
        cyc = c["GRBM_GUI_ACTIVE"] / XCDS
        n_mfma = c["SQ_INSTS_VALU_MFMA_MOPS_I8"] / MOPS_PER_MFMA
        wc = c["SQ_WAVE_CYCLES"]
        res[k] = {
            "launches_averaged": cnt[k],
            "kernel_cycles": cyc,
            "mfma_busy": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc),
            "n_mfma": n_mfma,
            "valu_per_mfma": c["SQ_INSTS_VALU"] / n_mfma,
            "salu_per_mfma": c["SQ_INSTS_SALU"] / n_mfma,
            "lds_per_mfma": c["SQ_INSTS_LDS"] / n_mfma,
            "smem_per_mfma": c["SQ_INSTS_SMEM"] / n_mfma,
            "wave_wait_any": c["SQ_WAIT_ANY"] / wc,
            "wave_wait_inst_any": c["SQ_WAIT_INST_ANY"] / wc,
            "wave_active_inst_any": c["SQ_ACTIVE_INST_ANY"] / wc,
            "simd_valu_active": c["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc),
            "simd_salu_active": c["SQ_ACTIVE_INST_SCA"] * 4 / (SIMDS * cyc),
            "simd_lds_active": c["SQ_ACTIVE_INST_LDS"] * 4 / (SIMDS * cyc),
            "wait_inst_lds_frac": c["SQ_WAIT_INST_LDS"] / wc,
            "raw": c,
        }
    json.dump(res, open(out, "w"), indent=1)
    for k in kinds:
        if k in res:
            r = res[k]
            print(f"{label} {k}: {r['kernel_cycles']:.3g} cyc, MFMA busy {r['mfma_busy']:.3f}, per MFMA: VALU "
                  f"{r['valu_per_mfma']:.2f} SALU {r['salu_per_mfma']:.2f} LDS {r['lds_per_mfma']:.2f}; waves: parked "
                  f"{r['wave_wait_any']:.2f} issue-stalled {r['wave_wait_inst_any']:.2f} issuing "
                  f"{r['wave_active_inst_any']:.2f}; SIMD VALU {r['simd_valu_active']:.2f} SALU "
                  f"{r['simd_salu_active']:.2f}")


if __name__ == "__main__":
    main()
