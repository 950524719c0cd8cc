#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel totals for the prefill window (first to
last prefill kernel), for the decode phase and per decode step.

The decode window is cut from the trace itself. Every decode step samples exactly once
(sample_final_kernel) after one forward pass; the segments between consecutive sampling
dispatches after the LAST prefill kernel (flash-prefill attention, big-tile GEMM or a hipBLASLt
`Cijk` GEMM) are decode steps. A segment that holds more forward passes than a step (the
hipGraph capture's eager warm-up runs before the first replay) is skipped: the window starts
after the first segment whose decode-attention count is the per-step count (the most common
one, i.e. the layer count) and ends with the last sampling dispatch. The number of decode steps
is the number of sampling dispatches in the window; decode-attention dispatches / layers is
printed as a cross-check.

usage: python tools/prof_summary.py gpurun_out/prof_x/run_kernel_trace.csv|run_results.db [--layers 80] [--md out.md]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
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
    ap.add_argument("--layers", type=int, default=0, help="model layers (cross-check: attention calls / layers)")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    rows = load_rows(a.trace)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    is_prefill = lambda n: "attn_prefill" in n or "gemm_big" in n or "Cijk" in n   # noqa: E731
    is_sample = lambda n: "sample_final" in n                                          # noqa: E731
    last_prefill = max((i for i, r in enumerate(rows) if is_prefill(r["Kernel_Name"])), default=-1)
    samples = [i for i, r in enumerate(rows) if is_sample(r["Kernel_Name"]) and i > last_prefill]
    if len(samples) < 3:
        raise SystemExit("trace holds fewer than two decode steps after the last prefill kernel")
    first_prefill = min((i for i, r in enumerate(rows) if is_prefill(r["Kernel_Name"])), default=-1)
    pre_lines = []
    if first_prefill >= 0:
        pre = rows[first_prefill:last_prefill + 1]
        pagg = defaultdict(lambda: [0, 0.0])
        for r in pre:
            pagg[short(r["Kernel_Name"])][0] += 1
            pagg[short(r["Kernel_Name"])][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        ptot = sum(v[1] for v in pagg.values())
        pspan = (int(pre[-1]["End_Timestamp"]) - int(pre[0]["Start_Timestamp"])) / 1e3
        pre_lines = [f"prefill window (first to last prefill kernel; mixed steps include their decode rows): "
                     f"{len(pre)} dispatches, kernel time {ptot / 1e3:.2f} ms, wall span {pspan / 1e3:.2f} ms",
                     "", "| kernel | calls | total ms | % | avg us |", "|---|---|---|---|---|"]
        for k, (c, t) in sorted(pagg.items(), key=lambda kv: -kv[1][1])[:15]:
            pre_lines.append(f"| {k} | {c} | {t / 1e3:.3f} | {100 * t / ptot:.1f} | {t / c:.1f} |")
        pre_lines += ["", ""]
    attn = [sum(1 for j in range(a + 1, b) if "attn_decode" in rows[j]["Kernel_Name"])
            for a, b in zip(samples, samples[1:])]
    per_step = a.layers if a.layers in attn else max(set(attn), key=attn.count)
    first = next(i for i, n in enumerate(attn) if n == per_step)     # segment samples[i] -> samples[i+1]
    dec = rows[samples[first] + 1:samples[-1] + 1]
    steps = len(samples) - 1 - first
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
    lines.append("")
    lines.append(f"decode steps in the window: {steps} (sampling dispatches); per step: kernel time "
                 f"{tot / steps / 1e3:.3f} ms, wall span {span / steps / 1e3:.3f} ms, "
                 f"{len(dec) / steps:.1f} dispatches")
    full = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in dec
            if "attn_decode_kernel" in r["Kernel_Name"]]
    if full:
        lines.append(f"decode attention per call over the window: mean {sum(full) / len(full):.1f} us, "
                     f"median {sorted(full)[len(full) // 2]:.1f} us")
    if a.layers:
        n_attn = sum(c for k, (c, _) in agg.items() if "attn_decode" in k)
        lines.append(f"cross-check: {n_attn} decode-attention dispatches / {a.layers} layers = {n_attn / a.layers:.2f} steps")
    text = "\n".join(pre_lines + lines)
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
