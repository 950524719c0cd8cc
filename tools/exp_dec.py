#!/usr/bin/env python3
"""Decode-GEMM kernel-shape experiment: weight-streaming TB/s of selected plans across M for one
projection shape (weights rotated over >= 1 GiB so every call reads HBM).
usage: python tools/exp_dec.py [N K]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402

PLANS = {"tile64x128": [1, 3, 0, 2, 64, 128, 1], "tile128x128": [1, 2, 0, 2, 128, 128, 1],
         "tile128x256": [1, 3, 0, 2, 128, 256, 1],
         "dec128x224w8s4": [3, 4, 8, 8, 128, 224, 1], "dec128x224w8s3": [3, 3, 8, 8, 128, 224, 1],
         "dec128x256w8s3": [3, 3, 8, 8, 128, 256, 1], "dec128x256w4x2s3": [3, 3, 8, 4, 128, 256, 1],
         "dec128x128w8s5": [3, 5, 8, 8, 128, 128, 1], "dec128x128w4x2s5": [3, 5, 8, 4, 128, 128, 1],
         "dec64x128w4x2s6": [3, 6, 8, 4, 64, 128, 1], "dec64x256w4x2s4": [3, 4, 8, 4, 64, 256, 1]}


def bench(x, Ws, out, plan, ws, iters=20):
    f = lambda i: torch.ops.bfly.gemm_with_plan(x, Ws[i % len(Ws)], out, plan, 0, ws)  # noqa: E731
    for i in range(3):
        f(i)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for i in range(iters):
        f(i)
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


def main():
    assert ops.load_library()
    N, K = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (57344, 8192)
    ws = torch.zeros(64 << 20, dtype=torch.float32, device="cuda")
    copies = max(2, (1 << 30) // (N * K * 2) + 1)
    Ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
    for M in (32, 64, 128, 192, 256):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        row = {"N": N, "K": K, "M": M}
        for name, plan in PLANS.items():
            try:
                us = bench(x, Ws, out, plan, ws)
                row[name] = f"{us:.1f}us {N * K * 2 / us / 1e6:.2f}TB/s"
            except RuntimeError:
                row[name] = "n/a"
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
