#!/usr/bin/env python3
"""Decode GEMM seams (csrc/kernels/gemm.hip seam_*) in isolation: Llama-3-70B O (8192 x 8192,
split-K 8), down (8192 x 28672, split-K 4) and QKV (10240 x 8192) at M = 64, each as
  plain    linear(defer=True) + its separate consumer (rms_norm rows / rope_kv)
  seam     linear_rmsnorm_rows / linear_rope_kv (one launch)
  gemm     linear(defer=True) alone (the GEMM body's time)
Device time per call from CUDA events over N back-to-back calls. BFLY_SEAM_PROBE=1/2/3 in the
environment skips the seam's sibling wait / reduce (timing only: wrong results).
usage: python tools/seam_bench.py [--iters N]"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from butterfly_amd import ops  # noqa: E402
from butterfly_amd.ops import reference as ref  # noqa: E402


def timeit(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--M", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    M = a.M
    g = torch.Generator(device=dev).manual_seed(0)
    bf = lambda *s, sc=1.0: (torch.randn(*s, device=dev, generator=g) * sc).to(torch.bfloat16)  # noqa: E731
    out = {"M": M, "probe": int(os.environ.get("BFLY_SEAM_PROBE", "0")), "seam_xcd": os.environ.get("BFLY_SEAM_XCD", "1")}
    for name, N, K in (("o", 8192, 8192), ("down", 8192, 28672)):
        x, w, gam, res = bf(M, K), bf(N, K, sc=1 / math.sqrt(K)), bf(N), bf(M, N)
        out[name + "_gemm"] = timeit(lambda: ops.linear(x, w, defer=True), a.iters)
        out[name + "_plain"] = timeit(lambda: ops.rms_norm(ops.linear(x, w, defer=True), gam, 1e-5, residual=res, rows=True), a.iters)
        if ops.norm_seam_ok(M, N, K):
            out[name + "_seam"] = timeit(lambda: ops.linear_rmsnorm_rows(x, w, gam, 1e-5, res), a.iters)
    Hq, Hkv, D, H, BS = 64, 8, 128, 8192, 32
    N = (Hq + 2 * Hkv) * D
    x, w = bf(M, H), bf(N, H, sc=1 / math.sqrt(H))
    cos, sin = ref.rope_tables(D, 4096, 500000.0, device=dev)
    pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=dev)
    slots = torch.randperm(4 * M * BS, device=dev)[:M].to(torch.int32)
    kc = torch.zeros(4 * M, Hkv, BS, D, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros(4 * M, Hkv, D, BS, dtype=torch.bfloat16, device=dev)
    out["qkv_gemm"] = timeit(lambda: ops.linear(x, w, defer=True), a.iters)
    out["qkv_plain"] = timeit(lambda: ops.rope_kv(ops.linear(x, w, defer=True), pos, cos, sin, Hq, Hkv, slots, kc, vc), a.iters)
    if ops.norm_seam_ok(M, N, H, ops.SEAM_ROPE):
        out["qkv_seam"] = timeit(lambda: ops.linear_rope_kv(x, w, pos, cos, sin, Hq, Hkv, slots, kc, vc), a.iters)
    out["seam_error"] = ops.norm_seam_error(dev)
    print(json.dumps({k: round(v, 2) if isinstance(v, float) else v for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
