#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel totals for the decode phase (every
dispatch after the last prefill-attention dispatch) and per decode step.

usage: python tools/prof_summary.py gpurun_out/prof_x/run_kernel_trace.csv|run_results.db [--steps K] [--md out.md]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "")
    m = re.match(r"_ZN4bfly\d+(\w+?)I", n)
    if m:
        n = "bfly::" + m.group(1)
    return n[:70]


def load_rows(path: str) -> list:
    """Kernel dispatches from a rocprofv3 kernel-trace CSV or a rocpd SQLite database
    (rocprofv3's default output format on ROCm 7: `<name>_results.db`)."""
    if path.endswith(".db"):
        import sqlite3

        con = sqlite3.connect(path)
        return [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                for n, s, e in con.execute("select name, start, end from kernels")]
    return list(csv.DictReader(open(path)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=0, help="decode steps in the window (for per-step numbers)")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    rows = load_rows(a.trace)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the decode window starts after the prefill's last attention AND its trailing big-tile GEMMs
    last_prefill = max((i for i, r in enumerate(rows) if "attn_prefill" in r["Kernel_Name"]
                        or "gemm_big_kernel" in r["Kernel_Name"]), default=-1)
    dec = rows[last_prefill + 1:]
    agg = defaultdict(lambda: [0, 0.0])
    for r in dec:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += d
    tot = sum(v[1] for v in agg.values())
    span = (int(dec[-1]["End_Timestamp"]) - int(dec[0]["Start_Timestamp"])) / 1e3 if dec else 0
    lines = [f"decode window: {len(dec)} dispatches, kernel time {tot / 1e3:.2f} ms, wall span {span / 1e3:.2f} ms",
             "", "| kernel | calls | total ms | % | avg us |", "|---|---|---|---|---|"]
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| {k} | {c} | {t / 1e3:.3f} | {100 * t / tot:.1f} | {t / c:.1f} |")
    if a.steps:
        lines.append("")
        lines.append(f"per decode step (/{a.steps}): kernel time {tot / a.steps / 1e3:.3f} ms")
    text = "\n".join(lines)
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
