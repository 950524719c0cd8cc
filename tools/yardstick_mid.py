#!/usr/bin/env python3
"""Mid-M yardstick: our plan vs torch.matmul (hipBLASLt, measured only as a yardstick — no
GPU path of the framework calls it) at the tensor-parallel shard shapes, M = 128 / 256 / 512.

Each shape runs both sides back to back, weights rotated over >= 1 GiB of copies (every call
streams them from HBM). Under `rocprofv3 --kernel-trace` the library kernel names show which
macro tile / split (MT..x..x.., GSU) hipBLASLt picks for the shape; the script itself prints
event-timed microseconds per call (ours includes its split-K reduce launch).

usage: python tools/yardstick_mid.py [--shapes tp8,tp4] [--ms 128,256,512] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402
from tools.bench_gemm import SHAPES  # noqa: E402


def timed(fn, iters):
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
    ap.add_argument("--shapes", default="tp8,tp4")
    ap.add_argument("--ms", default="128,256,512")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    assert ops.load_library()
    for group in a.shapes.split(","):
        for name, N, K, epi in SHAPES[group]:
            if name == "lm_head":
                continue
            copies = max(2, (1 << 30) // (N * K * 2) + 1)
            Ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
            for M in (int(m) for m in a.ms.split(",")):
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                ours = timed(lambda i: ops.linear(x, Ws[i % copies], epilogue=epi), a.iters)
                lib = timed(lambda i: torch.matmul(x, Ws[i % copies].t()), a.iters)
                fl = 2.0 * M * N * K
                print(json.dumps({"shape": f"{group}.{name}", "M": M, "N": N, "K": K, "plan": ops.gemm_plan(M, N, K),
                                  "ours_us": round(ours, 2), "hipblaslt_us": round(lib, 2),
                                  "ours_TF": round(fl / ours / 1e6, 1), "hipblaslt_TF": round(fl / lib / 1e6, 1)}),
                      flush=True)


if __name__ == "__main__":
    main()
