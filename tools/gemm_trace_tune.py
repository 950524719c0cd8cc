#!/usr/bin/env python3
"""Pick GEMM plans from a serialised sweep profiled with rocprofv3 (per-dispatch durations,
no overlap between calls — what a GEMM costs inside a dependent decode chain).

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gt -o run -- \
      python3 tools/bench_gemm.py --sweep --serial gpurun_out/gt_log.jsonl ...
  python tools/gemm_trace_tune.py gpurun_out/gt/run_kernel_trace.csv gpurun_out/gt_log.jsonl \
      --out profiles/gemm_tune_<name>.json

Each logged candidate made `calls` GEMM calls; each call is one bfly GEMM dispatch plus, with
split-K, one reduce dispatch. The median over the timed calls (the first 3 are warm-up) of
(GEMM + reduce) is the candidate's cost. Output rows use bench_gemm.py's JSON schema so
tools/gen_gemm_table.py can consume them."""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("log")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if "gemm_" in r["Kernel_Name"] and "bfly" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cands = [json.loads(l) for l in open(a.log)]
    i = 0
    res = {}
    for c in cands:
        tag = c["tag"]
        sk = tag["plan"][6]
        costs = []
        for k in range(c["calls"]):
            r = rows[i]
            assert "reduce" not in r["Kernel_Name"], ("misaligned trace", i, tag)
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            i += 1
            if sk > 1 and i < len(rows) and "reduce" in rows[i]["Kernel_Name"]:
                d += int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])
                i += 1
            if k >= 3:
                costs.append(d / 1000.0)
        us = statistics.median(costs)
        key = (tag["shape"], tag["M"])
        e = res.setdefault(key, {"shape": tag["shape"], "M": tag["M"], "N": tag["N"], "K": tag["K"]})
        if tag.get("auto"):
            p = tag["plan"]
            e["plan"] = {"kind": ("skinny", "tile", "big", "dec", "big8", "mid8", "big4", "mid4")[p[0]], "mt": p[1], "nt": p[2], "wk": p[3],
                         "bm": p[4], "bn": p[5], "splitk": p[6]}
            e["us"] = round(us, 2)
            e["TBps"] = round(tag["N"] * tag["K"] * 2 / us / 1e6, 3)
        else:
            e.setdefault("cands", []).append([round(us, 2), tag["plan"]])
            if "best_us" not in e or us < e["best_us"]:
                e["best_us"], e["best_plan"] = round(us, 2), tag["plan"]
    assert i == len(rows), f"{len(rows) - i} unmatched dispatches"
    out = list(res.values())
    json.dump(out, open(a.out, "w"), indent=1)
    for e in out:
        print(f"{e['shape']:14s} M={e['M']:4d} auto {e['us']:7.1f}  best {e.get('best_us', 0):7.1f} {e.get('best_plan')}")


if __name__ == "__main__":
    main()
