#!/usr/bin/env python3
"""Is the M = 64 decode gate/up GEMM (Llama-3-70B: N = 57344 = 448 column tiles of 128, K = 8192)
bound by the uneven spread of its 448 workgroups over 256 CUs (192 CUs run two, 64 run one)?

Times the table's tile plan for the same K at N = 256 .. 512 tiles of 128 columns: if the time
tracks the tile count per CU (448 tiles as slow as 512) the kernel is bound per CU and a
balanced decomposition (stream-K over 256 workgroups) would pay; if it tracks the bytes, it
would not. Weight copies cycle through > 1 GiB so every call streams from HBM.

usage: python tools/balance_probe.py [--k 8192] [--m 64]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from butterfly_amd import ops  # noqa: E402


def timeit(fn, iters=20):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--m", type=int, default=64)
    a = ap.parse_args()
    assert ops.load_library()
    K, M = a.k, a.m
    plans = {"tile64x128_wk2": [1, 3, 0, 2, 64, 128, 1], "tile64x128_wk1": [1, 3, 0, 1, 64, 128, 1],
             "tile64x256_wk2": [1, 3, 0, 2, 64, 256, 1]}
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    for tiles in (256, 320, 384, 448, 512, 640, 768):
        N = tiles * 128
        nbytes = N * K * 2
        copies = max(2, (1 << 30) // nbytes + 1)
        Ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        out = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
        for name, pl in plans.items():
            if N % pl[5]:
                continue
            us = min(timeit(lambda i: torch.ops.bfly.gemm_with_plan(x, Ws[i % copies], out, pl, ops.EPILOGUES["silu"], None))
                     for _ in range(3))
            print(json.dumps({"plan": name, "M": M, "N": N, "K": K, "tiles": N // pl[5],
                              "tiles_per_cu": round(N / pl[5] / 256, 3), "us": round(us, 2),
                              "TBps": round(nbytes / us / 1e6, 3)}), flush=True)
        del Ws


if __name__ == "__main__":
    main()
