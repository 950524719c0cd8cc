#!/usr/bin/env python3
"""Markdown table of one rocprofv3 --pmc pass over tools/gemm_pmc.py: per kernel (mean over its
dispatches) GRBM_GUI_ACTIVE and the SQ counters, in millions, plus the MFMA-busy share computed
from the known MFMA work (QKV at M = 8192: 1.31 M cycles of 16x16x32 MFMA per SIMD).
usage: python tools/gemm_pmc_md.py gpurun_out/pmc_gemm/.../run_counter_collection.csv > out.md"""
import csv
import re
import sys
from collections import defaultdict

MFMA_CYCLES_PER_SIMD = 1.31e6


def short(n):
    if "gemm_big8_kernel" in n:
        return "gemm_big8_kernel"
    m = re.search(r"(Cijk_\w+?MT\w+?_MI\w+?)_", n)
    return ("hipBLASLt " + m.group(1)[:60]) if m else None


def main(path):
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k:
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    cols = ["GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_INSTS_VALU", "SQ_INSTS_LDS",
            "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS"]
    print("| kernel | " + " | ".join(c.replace("SQ_", "") for c in cols) + " | MFMA-busy % of cycles |")
    print("|---" * (len(cols) + 2) + "|")
    for k, d in vals.items():
        row = []
        for c in cols:
            v = d.get(c)
            row.append(f"{sum(v) / len(v) / 1e6:.2f}" if v else "-")
        g = d.get("GRBM_GUI_ACTIVE")
        busy = f"{100 * MFMA_CYCLES_PER_SIMD / (sum(g) / len(g) / 8):.0f}" if g else "-"
        print(f"| {k} | " + " | ".join(row) + f" | {busy} |")


if __name__ == "__main__":
    main(sys.argv[1])
