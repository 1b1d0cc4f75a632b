"""Summarise tools/pmc_x3.sh output: per counter, the median over the dispatches of the op's
kernel (the last dispatch name that is not a split/copy helper), plus derived ratios.

    python tools/pmc_summary.py gpurun_out/pmc_qkv_x3_cpx_t102 [...]
"""
from __future__ import annotations

import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def summarise(d: str) -> dict:
    vals = defaultdict(lambda: defaultdict(list))  # counter -> kernel -> values per dispatch
    for f in sorted(glob.glob(os.path.join(d, "p*_counter_collection.csv"))):
        per = defaultdict(float)
        names = {}
        with open(f) as fh:
            for row in csv.DictReader(fh):
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per[key] += float(row["Counter_Value"])
                names[row["Dispatch_Id"]] = row["Kernel_Name"]
        for (disp, cn), v in per.items():
            vals[cn][names[disp]].append(v)
    kernels = set()
    for cn in vals:
        kernels |= set(vals[cn])
    main = [k for k in kernels if "split3" not in k and "copy" not in k.lower() and "fill" not in k.lower()]
    out = {}
    for k in main:
        out[k] = {cn: statistics.median(v[k]) for cn, v in vals.items() if k in v}
    return out


def derived(c: dict) -> dict:
    r = {}
    g = lambda n: c.get(n, 0.0)  # noqa: E731
    if g("GRBM_GUI_ACTIVE"):
        r["gpu_cycles"] = g("GRBM_GUI_ACTIVE")
    if g("SQ_BUSY_CYCLES") and g("SQ_VALU_MFMA_BUSY_CYCLES"):
        r["mfma_busy_per_simd_cycle"] = g("SQ_VALU_MFMA_BUSY_CYCLES") / max(1.0, g("SQ_BUSY_CYCLES"))
    if g("SQ_WAVE_CYCLES"):
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VMEM", "SQ_INST_LEVEL_VMEM"):
            if n in c:
                r[f"{n}/WAVE_CYCLES"] = g(n) / g("SQ_WAVE_CYCLES")
    if g("TCC_HIT_sum") + g("TCC_MISS_sum"):
        r["l2_hit_rate"] = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    if g("SQ_LDS_IDX_ACTIVE"):
        r["lds_bank_conflict_frac"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")
    return r


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print("==", d)
        for k, c in summarise(d).items():
            print("  kernel:", k[:110])
            for cn in sorted(c):
                print(f"    {cn:34s} {c[cn]:.4g}")
            for n, v in derived(c).items():
                print(f"    -> {n:31s} {v:.4g}")
