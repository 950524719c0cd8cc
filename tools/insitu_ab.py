#!/usr/bin/env python3
"""Whole-step A/B of GEMM plan overrides against the plan table, alternating runs so a box's
drift (clocks, temperature: up to 0.4 ms on a 29 ms step within one call) hits both sides alike.

Each run is `bench.py` in its own process with BFLY_GEMM_PLAN set ("N,K,Mbucket:kind,mt,nt,wk,
bm,bn,sk"); for every candidate the sequence is base, cand, base, cand, ... (`--pairs` pairs) and
the report is the mean of (cand - preceding base) per pair, in ms per step.

usage: python tools/insitu_ab.py --model llama3-8b --pairs 3 \
           --cand "qA=6144,4096,64:1,4,0,2,64,128,4" --cand "d3=4096,14336,64:1,3,0,1,64,128,8"
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(model: str, plan: str, steps: int, out: str) -> float:
    env = dict(os.environ, BFLY_GEMM_PLAN=plan)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--model", model, "--steps", str(steps),
                        "--warmup", "4", "--out", out], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(f"bench failed ({r.returncode}): {r.stderr[-2000:]}")
    return json.loads(open(out).read().strip().splitlines()[-1])["ms_per_step"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--cand", action="append", default=[], help="tag=N,K,M:kind,mt,nt,wk,bm,bn,sk[;...]")
    ap.add_argument("--pairs", type=int, default=3)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--outdir", default="gpurun_out/insitu_ab")
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, a.outdir), exist_ok=True)
    for spec in a.cand:
        tag, plan = spec.split("=", 1)
        deltas, rows = [], []
        for i in range(a.pairs):
            b = run(a.model, "", a.steps, os.path.join(ROOT, a.outdir, f"{a.model}_base_{tag}_{i}.json"))
            c = run(a.model, plan, a.steps, os.path.join(ROOT, a.outdir, f"{a.model}_{tag}_{i}.json"))
            deltas.append(c - b)
            rows.append([round(b, 3), round(c, 3)])
            print(json.dumps({"model": a.model, "cand": tag, "pair": i, "base_ms": b, "cand_ms": c}), flush=True)
        print(json.dumps({"model": a.model, "cand": tag, "plan": plan, "pairs": rows,
                          "mean_delta_ms": round(statistics.mean(deltas), 3),
                          "max_delta_ms": round(max(deltas), 3)}), flush=True)


if __name__ == "__main__":
    main()
