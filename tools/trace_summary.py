#!/usr/bin/env python3
"""Summarise chrome traces written with BFLY_TRACE: per event name, count / total / median /
max duration (ms), per file (rank). Used to show where the host waits inside engine ticks.
usage: python tools/trace_summary.py trace_rank0.json [trace_rank1.json ...] [--md out.md]"""
import argparse
import json
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("traces", nargs="+")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    lines = []
    for path in a.traces:
        ev = json.load(open(path))["traceEvents"]
        by = defaultdict(list)
        for e in ev:
            by[e["name"]].append(e["dur"] / 1e3)
        lines += [f"### {path}", "", "| range | count | total ms | median ms | max ms |", "|---|---|---|---|---|"]
        for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            lines.append(f"| {name} | {len(d)} | {sum(d):.2f} | {statistics.median(d):.3f} | {max(d):.3f} |")
        lines.append("")
    text = "\n".join(lines)
    print(text)
    if a.md:
        open(a.md, "w").write(text + "\n")


if __name__ == "__main__":
    main()
