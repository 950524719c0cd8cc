#!/usr/bin/env python3
"""Routed-expert FFN microbenchmark (ops.moe_sparse_ffn: align, grouped gate/up GEMM with fused
SiLU, grouped down GEMM, weighted combine) at Mixtral 8x7B dimensions.

Reports the whole op's time and the useful GEMM FLOPs over it (2 * rows * H * 2ffn + 2 * rows *
ffn * H for the routed rows only), so the TF/s figure is a lower bound on the grouped GEMMs'
own rate. `--skew` routes a share of the tokens to expert 0 (uneven tiles, empty experts).

usage: python tools/bench_moe.py [--tokens 16384,4096,512] [--experts 8] [--topk 2] [--skew 0.0]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402
from tools.bench_attn import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="16384,4096,512")
    ap.add_argument("--experts", type=int, default=8)
    ap.add_argument("--topk", type=int, default=2)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--ffn", type=int, default=14336)
    ap.add_argument("--skew", type=float, default=0.0, help="share of tokens whose first choice is expert 0")
    a = ap.parse_args()
    assert torch.cuda.is_available() and ops.load_library(), "needs a GPU and the built kernels"
    E, H, F, k = a.experts, a.hidden, a.ffn, a.topk
    g = torch.Generator(device="cuda").manual_seed(0)
    gu = (torch.randn(E * 2 * F, H, device="cuda", generator=g) * 0.02).bfloat16()
    dn = (torch.randn(H, E * F, device="cuda", generator=g) * 0.02).bfloat16()
    for T in map(int, a.tokens.split(",")):
        x = torch.randn(T, H, device="cuda", generator=g).bfloat16()
        ids = torch.stack([torch.randperm(E, device="cuda", generator=g)[:k] for _ in range(T)]).int()
        if a.skew > 0:
            n0 = int(a.skew * T)
            ids[:n0, 0] = 0
            ids[:n0, 1:] = torch.where(ids[:n0, 1:] == 0, 1, ids[:n0, 1:])
        w = torch.softmax(torch.randn(T, k, device="cuda", generator=g), -1)
        f = lambda: ops.moe_sparse_ffn(x, ids, w, gu, dn, 0, E, F)  # noqa: E731
        us = timed(f)
        flops = 2.0 * T * k * H * 2 * F + 2.0 * T * k * F * H
        print(json.dumps({"tokens": T, "routed_rows": T * k, "experts": E, "skew": a.skew, "us": round(us, 1),
                          "TFLOPs_useful": round(flops / us / 1e6, 1),
                          "tile_rows": 256 if T * k >= 256 * E else (128 if T * k >= 96 * E else 64)}), flush=True)


if __name__ == "__main__":
    main()
