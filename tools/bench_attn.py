#!/usr/bin/env python3
"""Paged decode-attention microbenchmark (KV bytes streamed per call -> TB/s)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="64:1024:64:8,64:1024:8:1,256:1024:64:8,1:8192:64:8,16:4096:64:8")
    a = ap.parse_args()
    ops.load_library()
    for case in a.cases.split(","):
        B, ctx, Hq, Hkv = map(int, case.split(":"))
        D, BS = 128, 32
        nb = (ctx + BS - 1) // BS
        kc = torch.randn(B * nb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn(B * nb, Hkv, D, BS, device="cuda", dtype=torch.bfloat16)
        bt = torch.randperm(B * nb, device="cuda").to(torch.int32).view(B, nb)
        cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
        out = torch.empty_like(q)
        f = lambda: ops.attn_decode(q, kc, vc, bt, cl, 0.088, ctx, out=out)  # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        st.record()
        for _ in range(it):
            f()
        en.record()
        torch.cuda.synchronize()
        us = st.elapsed_time(en) / it * 1e3
        byts = 2 * B * ctx * Hkv * D * 2
        print(json.dumps({"B": B, "ctx": ctx, "Hq": Hq, "Hkv": Hkv, "us": round(us, 2),
                          "TBps": round(byts / us / 1e6, 3),
                          "part_tokens": torch.ops.bfly.attn_decode_part_tokens(B, Hkv, ctx)}), flush=True)


if __name__ == "__main__":
    main()
