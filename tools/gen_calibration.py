#!/usr/bin/env python3
"""Regenerate partition/calibration/mi355x_gemm.json (the cost model's GEMM times) from the
serialised plan sweeps (profiles/gemm_tune_*.json): per (N, K, M-bucket) the fastest measured
plan, i.e. what plan_gemm() runs (its table holds those winners). Entries listed under
"in_situ" keep their in-step kernel times."""
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAL = os.path.join(ROOT, "butterfly_amd", "partition", "calibration", "mi355x_gemm.json")


def main():
    old = json.load(open(CAL))
    keep = set(old.get("in_situ", {}).get("keys", []))
    best = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "gemm_tune_*.json"))):
        for r in json.load(open(f)):
            key = f"{r['N']}x{r['K']}x{r['M']}"
            cands = [us for us, _ in r.get("cands", [])]
            if r.get("us") == r.get("us") and r.get("us"):   # the auto plan (not NaN)
                cands.append(r["us"])
            if cands:
                best[key] = min(best.get(key, 1e30), min(cands))
    # round-6 event-timed same-run sweeps (the plan table takes their winners): best candidate
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r6_gemm", "sweep_evt_*.json"))):
        for r in json.load(open(f)):
            if r.get("best_us"):
                key = f"{r['N']}x{r['K']}x{r['M']}"
                best[key] = min(best.get(key, 1e30), r["best_us"])
    gemm = dict(old.get("gemm", {}))
    n = 0
    for key, us in best.items():
        if key in keep:
            continue
        gemm[key] = round(us, 2)
        n += 1
    old["gemm"] = dict(sorted(gemm.items()))
    old["source"] = ("tools/gen_calibration.py: fastest plan per shape in profiles/gemm_tune_*.json (rocprofv3-"
                     "serialised sweeps) and profiles/r6_gemm/sweep_evt_*.json (event-timed same-run sweeps)")
    json.dump(old, open(CAL, "w"), indent=1)
    print(f"{n} entries updated, {len(gemm)} total")


if __name__ == "__main__":
    main()
