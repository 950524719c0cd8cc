#!/usr/bin/env python3
"""Time explicit GEMM plans on one projection shape, weights streamed from HBM (rotating copies
>= 1 GiB, like a decode step that touches 80 layers in between). Split-K plans run with their
reduce kernel; the reduce alone is timed too, so GEMM-only time = total - reduce.

usage: python tools/exp_plans.py --n 10240 --k 8192 --m 64 --plans "1,2,0,4,64,160,8;3,6,8,4,64,128,3"
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402


def timeit(fn, iters=40):
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
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--k", type=int, required=True)
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--epi", default="none")
    ap.add_argument("--plans", required=True)
    a = ap.parse_args()
    assert ops.load_library()
    N, K, M = a.n, a.k, a.m
    copies = max(2, (1 << 30) // (N * K * 2) + 1)
    Ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(M, N // 2 if a.epi == "silu" else N, device="cuda", dtype=torch.bfloat16)
    ws = torch.zeros(64 << 20, dtype=torch.float32, device="cuda")
    auto = ops.gemm_plan(M, N, K)
    print(f"shape N={N} K={K} M={M} auto plan {auto}", flush=True)
    for spec in a.plans.split(";"):
        pl = [int(v) for v in spec.split(",")]
        try:
            t = timeit(lambda i: torch.ops.bfly.gemm_with_plan(x, Ws[i % copies], out, pl, ops.EPILOGUES[a.epi], ws))
        except RuntimeError as e:
            print(f"plan {pl}: rejected ({str(e).splitlines()[0]})", flush=True)
            continue
        sk = pl[6]
        tr = 0.0
        if sk > 1:
            slabs = torch.zeros(sk, M, N, dtype=torch.float32, device="cuda")
            o2 = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            tr = timeit(lambda i: torch.ops.bfly.splitk_reduce(slabs, o2))
        g = t - tr
        print(f"plan {pl}: total {t:.2f} us, reduce {tr:.2f} us, gemm {g:.2f} us = {N * K * 2 / g / 1e6:.2f} TB/s",
              flush=True)


if __name__ == "__main__":
    main()
