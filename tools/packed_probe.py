#!/usr/bin/env python3
"""Decode gate/up GEMM (M = 64) over a K-tile-blocked weight layout [N/256][K/64][256][64]
against the row-major weight: same tile plan, same arithmetic order (outputs bitwise equal),
different DRAM access pattern (a 128-row stage reads one 16 KiB run instead of 128 runs of
128 B one row pitch apart). Weight copies rotate over > 1 GiB so every call streams from HBM.

usage: python tools/packed_probe.py [--n 57344] [--k 8192] [--m 64]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from butterfly_amd import ops  # noqa: E402


def pack_w256(w: torch.Tensor) -> torch.Tensor:
    N, K = w.shape
    return w.view(N // 256, 256, K // 64, 64).permute(0, 2, 1, 3).contiguous().view(N, K)


def timeit(fn, iters=30):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for i in range(iters):
        fn(i)
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


def table_plan(M, N, K):
    p = ops.gemm_plan(M, N, K)
    kinds = ("skinny", "tile", "big", "dec", "big8", "mid8", "big4", "mid4")
    return [kinds.index(p["kind"]), p["mt"], p["nt"], p["wk"], p["bm"], p["bn"], p["splitk"]]


def split_k_shapes(M):
    """The table plans of the other decode projections, row-major vs packed (split-K plans,
    their reduce launch included)."""
    ws = torch.zeros(256 << 20, dtype=torch.float32, device="cuda")
    for name, N, K in (("70b.qkv", 10240, 8192), ("70b.o", 8192, 8192), ("70b.down", 8192, 28672),
                       ("8b.down", 4096, 14336), ("mixtral.moe_down", 4096, 114688)):
        pl = table_plan(M, N, K)
        if pl[0] != 1 or pl[4] != 64:
            continue
        copies = max(2, (1 << 30) // (N * K * 2) + 1)
        Ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        Ps = [pack_w256(w) for w in Ws]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        pk = list(pl)
        pk[2] = 1
        for rep in range(2):
            for case, W, p in (("rowmajor", Ws, pl), ("packed", Ps, pk)):
                us = timeit(lambda i: torch.ops.bfly.gemm_with_plan(x, W[i % copies], out, p, 0, ws))
                print(json.dumps({"rep": rep, "shape": name, "case": case, "plan": p, "us": round(us, 2),
                                  "TBps": round(N * K * 2 / us / 1e6, 3)}), flush=True)
        del Ws, Ps


SWEEP_SHAPES = {"70b.qkv": (10240, 8192, "none"), "70b.o": (8192, 8192, "none"), "70b.down": (8192, 28672, "none"),
                "70b.gate_up": (57344, 8192, "silu"), "8b.qkv": (6144, 4096, "none"), "8b.o": (4096, 4096, "none"),
                "8b.gate_up": (28672, 4096, "silu"), "8b.down": (4096, 14336, "none")}


def sweep(M, names):
    """Every packed tile plan (64-row tiles; 128 / 256 columns, 1 / 2 waves along M, 2-4 stages,
    split-K 1-8) against the table plan on the row-major and the packed weight, event-timed with
    the weights rotating through HBM; split-K plans include their reduce launch."""
    ws = torch.zeros(256 << 20, dtype=torch.float32, device="cuda")
    for name in names:
        N, K, e = SWEEP_SHAPES[name]
        epi = ops.EPILOGUES[e]
        copies = max(2, (1 << 30) // (N * K * 2) + 1)
        Ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        Ps = [pack_w256(w) for w in Ws]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(M, N // 2 if e == "silu" else N, device="cuda", dtype=torch.bfloat16)
        tp = table_plan(M, N, K)
        cands = [("table_rowmajor", Ws, tp)]
        if tp[0] == 1 and tp[4] <= 64:
            cands.append(("table_packed", Ps, tp[:2] + [1] + tp[3:]))
        for bn in (128, 256):
            for wk in (1, 2):
                for st in (2, 3, 4):
                    for sk in (1, 2, 3, 4, 6, 8):
                        if (K // 64) < 4 * sk:
                            continue
                        cands.append((f"packed_{bn}_{wk}_{st}_{sk}", Ps, [1, st, 1, wk, 64, bn, sk]))
        res = {}
        for rep in range(2):
            for tag, W, pl in cands:
                try:
                    us = timeit(lambda i: torch.ops.bfly.gemm_with_plan(x, W[i % copies], out, pl, epi, ws), iters=20)
                except RuntimeError:
                    continue
                res.setdefault(tag, []).append(us)
        best = sorted((min(v), k) for k, v in res.items())
        for us, tag in best[:6] + [(min(res["table_rowmajor"]), "table_rowmajor")]:
            print(json.dumps({"shape": name, "M": M, "case": tag, "us": round(us, 2),
                              "TBps": round(N * K * 2 / us / 1e6, 3), "table_plan": tp}), flush=True)
        del Ws, Ps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=57344)
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--others", action="store_true", help="also the split-K decode projections")
    ap.add_argument("--sweep", default="", help="comma-separated SWEEP_SHAPES names: sweep packed tile plans")
    a = ap.parse_args()
    assert ops.load_library()
    N, K, M = a.n, a.k, a.m
    if a.sweep:
        sweep(M, a.sweep.split(","))
        return
    if a.others:
        split_k_shapes(M)
        return
    copies = max(2, (1 << 30) // (N * K * 2) + 1)
    Ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
    Ps = [pack_w256(w) for w in Ws]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    ref = torch.empty_like(out)
    silu = ops.EPILOGUES["silu"]
    torch.ops.bfly.gemm_with_plan(x, Ws[0], ref, [1, 3, 0, 2, 64, 128, 1], silu, None)
    torch.ops.bfly.gemm_with_plan(x, Ps[0], out, [1, 3, 1, 2, 64, 128, 1], silu, None)
    torch.cuda.synchronize()
    print(json.dumps({"bitwise_equal": bool(torch.equal(out, ref))}), flush=True)
    cases = [("rowmajor_wk2", Ws, [1, 3, 0, 2, 64, 128, 1]), ("packed_wk2", Ps, [1, 3, 1, 2, 64, 128, 1]),
             ("rowmajor_wk1", Ws, [1, 3, 0, 1, 64, 128, 1]), ("packed_wk1", Ps, [1, 3, 1, 1, 64, 128, 1])]
    for rep in range(3):
        for name, W, pl in cases:
            us = timeit(lambda i: torch.ops.bfly.gemm_with_plan(x, W[i % copies], out, pl, silu, None))
            print(json.dumps({"rep": rep, "case": name, "M": M, "N": N, "K": K, "us": round(us, 2),
                              "TBps": round(N * K * 2 / us / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
