#!/usr/bin/env python3
"""Experiment: does reading a projection's weights shortly before the GEMM (so they sit in the
256 MiB Infinity Cache / L2) shorten the decode GEMM? Measures each GEMM alone with events,
(a) cold: weights rotated over >= 1 GiB of copies, (b) after a full read of the same weights,
(c) after a prefetch kernel on a second stream that overlaps a latency-bound kernel chain.

usage: python tools/exp_prefetch.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402


def main():
    assert ops.load_library(), ops._load_error
    dev = torch.device("cuda:0")
    M = 64
    for name, N, K in (("o", 8192, 8192), ("qkv", 10240, 8192)):
        ncopy = max(2, (1 << 30) // (N * K * 2) + 1)
        Ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        res = {"shape": name, "N": N, "K": K, "M": M, "MB": N * K * 2 / 1e6}
        side = torch.cuda.Stream()
        sink = torch.empty(1, device=dev, dtype=torch.float32)
        for mode in ("cold", "touched", "touched_nt_gap", "overlap_prefetch"):
            ts = []
            for it in range(3 * ncopy):
                W = Ws[it % ncopy]
                if mode == "touched":
                    torch.sum(W.view(torch.int32), dtype=torch.int64)
                elif mode == "touched_nt_gap":
                    torch.sum(W.view(torch.int32), dtype=torch.int64)
                    # a different 256 MiB read in between: is the cache then cold again?
                    torch.sum(Ws[(it + 1) % ncopy].view(torch.int32)[: N // 2], dtype=torch.int64)
                elif mode == "overlap_prefetch":
                    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                    ev = torch.cuda.Event()
                    ev.record()
                    side.wait_event(ev)
                    with torch.cuda.stream(side):
                        torch.sum(W.view(torch.int32), dtype=torch.int64)
                    for _ in range(10):        # small latency-bound kernels on the main stream
                        a = a * 1.0001
                    torch.cuda.current_stream().wait_stream(side)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.linear(x, W)
                e1.record()
                torch.cuda.synchronize()
                if it >= ncopy:
                    ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            res[mode + "_us"] = round(ts[len(ts) // 2], 1)
        # how long does the touch itself take?
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(ncopy):
            torch.sum(Ws[i].view(torch.int32), dtype=torch.int64)
        e1.record()
        torch.cuda.synchronize()
        res["touch_us"] = round(e0.elapsed_time(e1) * 1e3 / ncopy, 1)
        sink.zero_()
        print(json.dumps(res), flush=True)
        del Ws


if __name__ == "__main__":
    main()
