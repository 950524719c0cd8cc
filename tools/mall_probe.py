#!/usr/bin/env python3
"""Does the Infinity Cache (MALL, 256 MB memory-side) speed up a decode GEMM whose weights
were read shortly before? Llama-3-70B decode projections at B=64 (split-K deferred, as in
the decode step), timed three ways, each after a 1 GiB flush:

  cold      flush -> GEMM
  warm      GEMM -> GEMM (whole weight read once just before)
  pre<f>    flush -> read the first f of every split-K chunk of every weight row -> GEMM

If `warm` is much faster than `cold`, prefetching the next GEMM's weights during the
latency-bound norm / rope kernels (HBM idle there) pays.

usage: python tools/mall_probe.py [--reps 10]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402

SHAPES = [("qkv", 10240, 8192), ("o", 8192, 8192), ("down", 8192, 28672)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    assert ops.load_library(), ops._load_error
    flush = torch.zeros(256 << 20, dtype=torch.float32, device="cuda")
    M = 64
    for name, N, K in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.02).to(torch.bfloat16)
        sk = ops.gemm_plan(M, N, K)["splitk"]
        wv = w.view(N, sk, K // sk)

        def gemm():
            return ops.linear(x, w, defer=True)

        def timed(pre):
            ts = []
            for _ in range(a.reps):
                flush.add_(1.0)
                if pre is not None:
                    pre()
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                gemm()
                en.record()
                torch.cuda.synchronize()
                ts.append(st.elapsed_time(en) * 1e3)
            return round(statistics.median(ts), 1)

        gemm()
        torch.cuda.synchronize()
        row = {"shape": name, "N": N, "K": K, "sk": sk, "weight_MB": round(N * K * 2 / 1e6, 1),
               "cold_us": timed(None), "warm_us": timed(gemm)}
        for f in (0.1, 0.25, 0.5):
            cut = max(8, int(K // sk * f) // 8 * 8)
            row[f"pre{f}_us"] = timed(lambda: torch.amax(wv[:, :, :cut]))
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
