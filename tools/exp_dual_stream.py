#!/usr/bin/env python3
"""Experiment: can the decode step's kernel boundaries be hidden by running the batch as two
half-batches on two streams (each half's kernel ramp / tail overlaps the other half's steady
streaming, and the second reader of a weight panel hits L2 / the Infinity Cache)?

A 70B-shaped layer chain (add+RMSNorm, QKV, RMSNorm, O, add+RMSNorm, gate/up, down) over
`--layers` distinct weight sets (1.76 GB each, so nothing stays cached across layers) is timed
  single64  one stream, M = 64 (the engine today)
  single32  one stream, M = 32 (what one half costs alone)
  dual      two streams, M = 32 each, launched together
  dual_lag  two streams, the second starts one kernel behind the first
  graph_*   the same captured into one hipGraph (fork / join events), replayed
Each mode reports the median ms per layer over `--iters` chains. Split-K GEMM workspaces are
per stream (the counters and slabs of concurrent GEMMs must not alias).

usage: python tools/exp_dual_stream.py [--layers 8] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402

H, QKV, FFN = 8192, 10240, 28672


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    assert ops.load_library(), ops._load_error
    dev = torch.device("cuda:0")
    L = a.layers

    def w(n, k):
        return torch.empty(n, k, device=dev, dtype=torch.bfloat16).normal_(0, 0.02)

    layers = [dict(qkv=w(QKV, H), o=w(H, H), gu=w(2 * FFN, H), d=w(H, FFN), g1=torch.ones(H, device=dev, dtype=torch.bfloat16),
                   g2=torch.ones(H, device=dev, dtype=torch.bfloat16)) for _ in range(L)]
    shapes = ((QKV, H), (H, H), (2 * FFN, H), (H, FFN))

    def ws_for(M):
        need = max(torch.ops.bfly.gemm_workspace_size(M, n, k) for n, k in shapes)
        return torch.zeros(need // 4 + 1, device=dev, dtype=torch.float32)

    class Half:
        def __init__(self, M):
            self.M = M
            self.x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
            self.res = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
            self.y = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
            self.qkv = torch.empty(M, QKV, device=dev, dtype=torch.bfloat16)
            self.o = torch.empty(M, H, device=dev, dtype=torch.bfloat16)
            self.gu = torch.empty(M, FFN, device=dev, dtype=torch.bfloat16)
            self.ws = ws_for(M)

        def kernels(self, lw):
            """The layer as a list of launch thunks (so two halves can be interleaved)."""
            g = torch.ops.bfly
            return [
                lambda: g.rms_norm(self.x, lw["g1"], 1e-5, self.y, self.res),
                lambda: g.gemm(self.y, lw["qkv"], self.qkv, None, 0, self.ws),
                lambda: g.rms_norm(self.x, lw["g1"], 1e-5, self.y, None),   # stands in for rope / attention
                lambda: g.gemm(self.y, lw["o"], self.o, None, 0, self.ws),
                lambda: g.rms_norm(self.o, lw["g2"], 1e-5, self.y, self.res),
                lambda: g.gemm(self.y, lw["gu"], self.gu, None, ops.EPILOGUES["silu"], self.ws),
                lambda: g.gemm(self.gu, lw["d"], self.x, None, 0, self.ws),
            ]

    s_side = torch.cuda.Stream()
    h64, ha, hb = Half(64), Half(32), Half(32)

    def single(h):
        for lw in layers:
            for k in h.kernels(lw):
                k()

    def dual(lag):
        s_main = torch.cuda.current_stream()   # the capture stream under graph capture
        ev = torch.cuda.Event()
        ev.record(s_main)
        s_side.wait_event(ev)
        ka = [k for lw in layers for k in ha.kernels(lw)]
        kb = [k for lw in layers for k in hb.kernels(lw)]
        # issue order only: each stream runs its own chain; `lag` holds stream b back by one
        # kernel of stream a
        if lag:
            ka[0]()
            evl = torch.cuda.Event()
            evl.record(s_main)
            s_side.wait_event(evl)
            ka = ka[1:]
        with torch.cuda.stream(s_side):
            for k in kb:
                k()
        for k in ka:
            k()
        s_main.wait_stream(s_side)

    def timed(fn):
        ts = []
        for it in range(a.iters + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(e0.elapsed_time(e1) / L)
        ts.sort()
        return round(ts[len(ts) // 2], 4)

    def graphed(fn):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        torch.cuda.synchronize()
        return timed(g.replay)

    res = {"layers": L, "layer_weight_GB": round(sum(n * k for n, k in shapes) * 2 / 1e9, 3)}
    res["single64_ms"] = timed(lambda: single(h64))
    res["single32_ms"] = timed(lambda: single(ha))
    res["dual_ms"] = timed(lambda: dual(False))
    res["dual_lag_ms"] = timed(lambda: dual(True))
    print(json.dumps(res), flush=True)
    res["graph_single64_ms"] = graphed(lambda: single(h64))
    print(json.dumps(res), flush=True)
    try:
        res["graph_dual_ms"] = graphed(lambda: dual(False))
        res["graph_dual_lag_ms"] = graphed(lambda: dual(True))
    except Exception as e:  # noqa: BLE001
        res["graph_dual_error"] = repr(e)[:200]
    # two graphs (one per half) replayed on two streams: concurrency that does not depend on
    # the runtime running one graph's parallel branches together
    try:
        single(ha)
        single(hb)
        torch.cuda.synchronize()
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga):
            single(ha)
        with torch.cuda.graph(gb):
            single(hb)
        torch.cuda.synchronize()

        def two_graphs():
            cur = torch.cuda.current_stream()
            ev = torch.cuda.Event()
            ev.record(cur)
            s_side.wait_event(ev)
            ga.replay()
            with torch.cuda.stream(s_side):
                gb.replay()
            cur.wait_stream(s_side)

        res["two_graphs_ms"] = timed(two_graphs)
    except Exception as e:  # noqa: BLE001
        res["two_graphs_error"] = repr(e)[:200]
    # HBM floor of one layer's weights at 6.3 TB/s
    res["floor_ms_at_6.3TBps"] = round(res["layer_weight_GB"] / 6.3, 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
