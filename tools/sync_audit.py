#!/usr/bin/env python3
"""Host-synchronisation audit of engine steps from a rocprofv3 HIP runtime trace.

Input: a directory written by `rocprofv3 --kernel-trace --hip-runtime-trace --marker-trace
--output-format csv` of a run with BFLY_ROCTX=1 (every `LLMEngine.step` is an `engine.step`
roctx range). For each step range after the first `--skip` ones (prefill, graph capture), the
HIP API calls made by the stepping thread inside the range are classified:

* blocking: hipDeviceSynchronize, hipStreamSynchronize, hipEventSynchronize, hipMemcpy /
  hipMemcpyDtoH / hipMemcpyWithStream (the synchronous copies behind torch's `.item()` /
  `.tolist()` of a device tensor) — the host waits for the device;
* async: everything else (launches, graph replays, hipMemcpyAsync, event records).

A hipEventSynchronize on an event that completed long ago returns in a few microseconds; the
report lists every blocking call with its duration so such waits are distinguishable from a
stall. Prints a markdown summary (and writes it with --md).

usage: python tools/sync_audit.py gpurun_out/prof_TAG/rank0 [--skip 4] [--md out.md]
"""
import argparse
import csv
import glob
import os
from collections import Counter, defaultdict

BLOCKING = ("hipDeviceSynchronize", "hipStreamSynchronize", "hipEventSynchronize", "hipMemcpy",
            "hipMemcpyDtoH", "hipMemcpyWithStream", "hipMemcpy2D", "hipCtxSynchronize")


def _rows(path):
    with open(path, newline="") as f:
        yield from csv.DictReader(f)


def _find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def audit(d, skip=4, marker="engine.step"):
    steps = []
    for r in _rows(_find(d, "marker_api_trace.csv")):
        if r.get("Function", "").startswith(marker):
            steps.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Thread_Id")))
    steps.sort()
    calls = defaultdict(list)       # thread -> [(start, end, function)]
    for r in _rows(_find(d, "hip_api_trace.csv")):
        calls[r.get("Thread_Id")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
    for v in calls.values():
        v.sort()
    out = []
    for i, (t0, t1, tid) in enumerate(steps):
        if i < skip:
            continue
        inside = [c for c in calls.get(tid, []) if t0 <= c[0] and c[1] <= t1]
        blocking = [(f, (e - s) / 1e3) for s, e, f in inside if f in BLOCKING]
        out.append({"step": i, "ms": (t1 - t0) / 1e6, "api_calls": len(inside),
                    "by_function": Counter(f for _, _, f in inside), "blocking": blocking})
    return out


def render(res, title):
    lines = [f"# {title}", "", "| step | step ms | HIP API calls | blocking calls (us) |", "|---|---|---|---|"]
    for r in res:
        b = ", ".join(f"{f} {us:.1f}" for f, us in r["blocking"]) or "none"
        lines.append(f"| {r['step']} | {r['ms']:.2f} | {r['api_calls']} | {b} |")
    tot = Counter()
    for r in res:
        tot.update(r["by_function"])
    lines += ["", "HIP API calls inside the audited steps, by function:", ""]
    lines += [f"* {f}: {n}" for f, n in tot.most_common()]
    worst = max((us for r in res for _, us in r["blocking"]), default=0.0)
    lines += ["", f"Longest blocking call inside an audited step: {worst:.1f} us."]
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=4, help="leading step ranges to leave out (prefill, capture)")
    ap.add_argument("--md", default=None)
    ap.add_argument("--title", default="Host synchronisation inside engine steps")
    a = ap.parse_args()
    md = render(audit(a.dir, a.skip), a.title)
    print(md)
    if a.md:
        with open(a.md, "w") as f:
            f.write(md)


if __name__ == "__main__":
    main()
