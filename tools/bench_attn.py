#!/usr/bin/env python3
"""Attention microbenchmark: causal flash prefill (TFLOP/s of useful causal FLOPs) and paged
decode (KV bytes streamed per call -> TB/s)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402


def timed(f, warm_ms=100.0, run_ms=200.0):
    """Mean microseconds per call: calls run back to back for >= warm_ms (clocks and caches
    settle; a handful of short calls is still on the idle clock) before >= run_ms are timed."""
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f()
    torch.cuda.synchronize()
    st.record()
    f()
    en.record()
    torch.cuda.synchronize()
    one = max(st.elapsed_time(en), 1e-3)
    for _ in range(max(2, int(warm_ms / one))):
        f()
    it = max(5, int(run_ms / one))
    st.record()
    for _ in range(it):
        f()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="64:1024:64:8,64:1024:8:1,256:1024:64:8,1:8192:64:8,16:4096:64:8")
    ap.add_argument("--prefill", default="16:1024:64:8,4:4096:64:8,1:16384:64:8",
                    help="prefill cases seqs:len:Hq:Hkv ('' to skip)")
    ap.add_argument("--noncausal", action="store_true", help="time the prefill cases without the causal mask")
    ap.add_argument("--parts", default="0", help="decode split sizes to try (0 = auto)")
    ap.add_argument("--kv-dtype", default="bf16,fp8", help="decode cache element types to time")
    ap.add_argument("--seq-tables", action="store_true", help="decode: each sequence's pages consecutive "
                    "(as the block manager hands them out to a fresh batch) instead of a random permutation")
    ap.add_argument("--rotate", type=int, default=1, help="decode: cycle through this many distinct caches "
                    "(>= 4 for a 1k-context B=64 cache: each call streams cold from HBM, as one layer of a step)")
    a = ap.parse_args()
    ops.load_library()
    for case in filter(None, "" if a.prefill == "none" else a.prefill.split(",")):
        n, Ls, Hq, Hkv = map(int, case.split(":"))
        D, T = 128, n * Ls
        q = torch.randn(T, Hq, D, device="cuda", dtype=torch.bfloat16)
        k = torch.randn(T, Hkv, D, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(T, Hkv, D, device="cuda", dtype=torch.bfloat16)
        cu = torch.arange(0, T + 1, Ls, dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        causal = not a.noncausal
        f = lambda: ops.attn_prefill(q, k, v, cu, Ls, 0.088, causal, out=out)  # noqa: E731
        us = timed(f)
        flops = 4.0 * n * Ls * Ls / (2 if causal else 1) * Hq * D   # useful FLOPs
        print(json.dumps({"prefill": case, "causal": causal, "us": round(us, 1),
                          "TFLOPs": round(flops / us / 1e6, 1)}), flush=True)
    for case, kvd in [(c, k) for c in filter(None, a.cases.split(",")) for k in filter(None, a.kv_dtype.split(","))]:
        B, ctx, Hq, Hkv = map(int, case.split(":"))
        cdt = torch.float8_e4m3fn if kvd == "fp8" else torch.bfloat16
        D, BS = 128, 32
        nb = (ctx + BS - 1) // BS
        kcs = [torch.randn(B * nb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16).to(cdt) for _ in range(a.rotate)]
        vcs = [torch.randn(B * nb, Hkv, D, BS, device="cuda", dtype=torch.bfloat16).to(cdt) for _ in range(a.rotate)]
        kc = kcs[0]
        turn = [0]
        bt = (torch.arange(B * nb, device="cuda") if a.seq_tables else torch.randperm(B * nb, device="cuda"))
        bt = bt.to(torch.int32).view(B, nb)
        cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
        out = torch.empty_like(q)
        for pt in [int(x) for x in a.parts.split(",")]:
            def f(pt=pt):
                i = turn[0] = (turn[0] + 1) % a.rotate
                ops.attn_decode(q, kcs[i], vcs[i], bt, cl, 0.088, ctx, part_tokens=pt, out=out)
            us = timed(f)
            byts = 2 * B * ctx * Hkv * D * kc.element_size()
            used = pt if pt > 0 else torch.ops.bfly.attn_decode_part_tokens(B, Hkv, ctx)
            print(json.dumps({"B": B, "ctx": ctx, "Hq": Hq, "Hkv": Hkv, "kv": kvd, "us": round(us, 2),
                              "TBps": round(byts / us / 1e6, 3), "part_tokens": used, "rotate": a.rotate}), flush=True)

if __name__ == "__main__":
    main()
