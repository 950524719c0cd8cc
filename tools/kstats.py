#!/usr/bin/env python3
"""Per-forward kernel breakdown of a rocprofv3 --kernel-trace CSV of tools/shard_bench.py (or
any run whose forwards each hold `layers` decode-attention dispatches): the last `--steps`
forwards (graph replays) are kept, and per kernel name the calls per forward, the median
duration and the time per forward are printed, plus the sum and the gaps between kernels.

usage: python tools/kstats.py run_kernel_trace.csv [--layers 80] [--steps 10] [--md out.md]
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "")).replace("void ", "")
    return n[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--layers", type=int, default=80)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--md", default=None)
    ap.add_argument("--grid", action="store_true", help="split kernels by grid size")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    att = [i for i, r in enumerate(rows) if "attn_decode_kernel" in r["Kernel_Name"]]
    per = a.layers
    # forward boundaries: every `per`-th decode attention starts a forward
    starts = att[::per]
    if len(starts) < a.steps + 1:
        raise SystemExit(f"only {len(starts)} forwards in the trace")
    first = starts[-a.steps - 1] if len(starts) > a.steps else starts[0]
    # a forward begins a few kernels before its first attention (embedding, norm, qkv): cut at
    # the kernel after the previous forward's last attention's layer tail: use start index of
    # the first kernel after the LM head of the previous forward ~ simpler: take the window
    # from the first attention of step 0 to the first attention of step `steps`, which is a
    # whole number of forwards shifted by a constant offset
    lo, hi = starts[-a.steps - 1], starts[-1]
    win = rows[lo:hi]
    agg = defaultdict(list)
    for r in win:
        key = short(r["Kernel_Name"])
        if a.grid:
            key += " grid " + str(r.get("Grid_Size_X", r.get("Grid_Size", "")))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    t0 = int(win[0]["Start_Timestamp"])
    t1 = int(rows[hi]["Start_Timestamp"])
    busy = sum(sum(v) for v in agg.values())
    wall = (t1 - t0) / 1e3
    lines = [f"window: {a.steps} forwards, {wall / a.steps:.1f} us per forward, kernels {busy / a.steps:.1f} us, "
             f"gaps {(wall - busy) / a.steps:.1f} us, {len(win) / a.steps:.0f} dispatches per forward", "",
             "| kernel | calls/fwd | median us | us/fwd | share |", "|---|---|---|---|---|"]
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {k} | {len(v) / a.steps:.1f} | {statistics.median(v):.2f} | {sum(v) / a.steps:.1f} | "
                     f"{sum(v) / busy * 100:.1f} % |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        open(a.md, "w").write(out + "\n")


if __name__ == "__main__":
    main()
