#!/usr/bin/env python3
"""Summarise tools/profile_counters.sh output (rocprofv3 --pmc CSVs) per bfly kernel:
duration, MFMA busy share, MFMA/LDS instruction counts, LDS bank conflicts, HBM bytes and
achieved bandwidth. Writes markdown (for profiles/).
usage: python tools/pmc_summary.py gpurun_out/pmc_sq gpurun_out/pmc_tcc --md profiles/x.md"""
import argparse
import csv
import re
from collections import defaultdict

NUM_CU = 256


def short(name):
    n = re.sub(r"\(.*", "", name).replace("void ", "")
    m = re.search(r"bfly::(\w+)<([^>]*)>", n)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.search(r"_ZN4bfly\d+(\w+?)I", n) or re.search(r"bfly::(?:\(anonymous namespace\)::)?(\w+)", n)
    return m.group(1) if m else None


def load(d):
    per = defaultdict(lambda: defaultdict(list))
    dur = {}
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = short(r["Kernel_Name"])
        if not k:
            continue
        did = r["Dispatch_Id"]
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[(k, did)] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    durs = defaultdict(list)
    for (k, _), v in dur.items():
        durs[k].append(v)
    return per, durs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sq")
    ap.add_argument("tcc")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    sq, dsq = load(a.sq)
    tcc, dtcc = load(a.tcc)
    lines = ["| kernel | us (median) | MFMA inst | MFMA TFLOP/s | % of 2.5 PF | MFMA busy (raw) | LDS inst | LDS bank-conflict cyc | FETCH MB |",
             "|---|---|---|---|---|---|---|---|---|"]
    for k in sorted(sq):
        c = sq[k]
        n = len(c.get("GRBM_GUI_ACTIVE", [1]))
        us = sorted(dsq[k])[len(dsq[k]) // 2]
        avg = lambda name: sum(c.get(name, [0])) / max(1, len(c.get(name, [1])))  # noqa: E731
        gui = avg("GRBM_GUI_ACTIVE")
        busy = avg("SQ_VALU_MFMA_BUSY_CYCLES")
        # MFMA busy cycles are summed over SIMDs (4 per CU); GUI_ACTIVE is chip cycles
        util = 100.0 * busy / max(1.0, gui * NUM_CU * 4)
        fetch_kb = sum(tcc.get(k, {}).get("FETCH_SIZE", [0])) / max(1, len(tcc.get(k, {}).get("FETCH_SIZE", [1])))
        tus = sorted(dtcc.get(k, [us]))[len(dtcc.get(k, [us])) // 2]
        mb = fetch_kb / 1024
        # every bfly MFMA is a 16x16x32 bf16 (16384 FLOP) except the prefill attention's 32x32x16 (32768)
        fl = 32768 if "attn_prefill" in k else 16384
        tf = avg("SQ_INSTS_MFMA") * fl / (us * 1e-6) / 1e12
        lines.append(f"| `{k}` | {us:.1f} | {avg('SQ_INSTS_MFMA'):.3g} | {tf:.0f} | {100 * tf / 2500:.1f} | {busy:.3g} | "
                     f"{avg('SQ_INSTS_LDS'):.3g} | {avg('SQ_LDS_BANK_CONFLICT'):.3g} | {mb:.1f} |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write("# rocprofv3 PMC counters per hot kernel (MI355X, Llama-3-70B shapes; tools/kernel_zoo.py)\n\n")
            f.write("Collected by `tools/profile_counters.sh` (two `--pmc` passes with `--kernel-trace` only). MFMA busy % = "
                    "MFMA TFLOP/s = SQ_INSTS_MFMA x FLOP per MFMA / kernel time (counts match M*N*K/(16*16*32) exactly "
                    "for the GEMMs); FETCH = TCC FETCH_SIZE, a relative number (it under-counts wide reads: "
                    "MI355X_MICROARCH.md).\n\n")
            f.write(out + "\n")


if __name__ == "__main__":
    main()
