#!/usr/bin/env python3
"""Prefill GEMM A/B on the Llama-3-70B projections: gemm_big8_kernel (plan kind 4: 8 waves,
8-phase BK 64) and gemm_big4_kernel (plan kind 6: one wave per SIMD, 128 x 128 wave tiles,
slot-fenced schedule) vs torch.matmul (hipBLASLt, yardstick only; not used by the framework).
The round-3 variants that lost are recorded in profiles/r3_gemm_prefill_pmc.md.

Random uniform [-1, 1) operands (cdna_hip_programming.md §5.4 rule 25: zero-filled data clocks
higher), interleaved rounds in one process (rule 24), median and min per variant. First checks
kinds 4 and 6 against the fp32 reference (M tail, split-K, bias and SiLU epilogues).

usage: python tools/bench_prefill_gemm.py [--ms 8192] [--rounds 5] [--check-only]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402
from butterfly_amd.ops import reference as ref  # noqa: E402

KINDS = (4, 6)   # 4: gemm_big8_kernel (8 waves, the default); 6: gemm_big4_kernel (one wave per SIMD)
SHAPES = [("qkv", 10240, 8192, "none"), ("o", 8192, 8192, "none"), ("gate_up", 57344, 8192, "silu"),
          ("down", 8192, 28672, "none")]


def uni(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def check(ws):
    """kind 4 vs the fp32 reference: M tails, split-K, bias and SiLU epilogues."""
    bad = []
    for kv, M, N, K, epi, sk in [(m,) + c for m in KINDS for c in [(256, 256, 128, "none", 1), (300, 512, 1024, "none", 1), (4097, 768, 640, "none", 1),
                             (1024, 1024, 2048, "silu", 1), (512, 1280, 4096, "none", 4), (777, 512, 1024, "bias", 1),
                             (2048, 2560, 8192, "none", 2)]]:
        kind, var = kv if isinstance(kv, tuple) else (kv, 0)
        x = uni(M, K) * 0.5
        w = uni(N, K) * 0.05
        b = uni(N) if epi == "bias" else None
        nout = N // 2 if epi == "silu" else N
        out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
        torch.ops.bfly.gemm_with_plan(x, w, out, [kind, var, 0, 0, 256, 256, sk], ops.EPILOGUES[epi], ws, b)
        want = ref.linear(x.float(), w.float(), b.float() if b is not None else None,
                          "silu" if epi == "silu" else "none")
        err = ((out.float() - want).abs() / (want.abs() + 2e-2)).max().item()
        rel = ((out.float() - want).norm() / want.norm()).item()
        row = {"kind": kind, "variant": var, "M": M, "N": N, "K": K, "epi": epi, "sk": sk, "max_rel_err": round(err, 4), "rel_l2": round(rel, 5)}
        print(json.dumps({"check": row}), flush=True)
        if rel > 1e-2:
            bad.append(row)
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="8192")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--sks", default="1", help="split-K factors tried per variant (best reported)")
    ap.add_argument("--variants", default="", help="comma list (default: all)")
    a = ap.parse_args()
    assert ops.load_library(), ops._load_error
    ws = torch.zeros(256 << 20, dtype=torch.float32, device="cuda")
    bad = check(ws)
    if bad or a.check_only:
        print(json.dumps({"check_failures": bad}), flush=True)
        return 1 if bad else 0
    for M in [int(m) for m in a.ms.split(",")]:
        for name, N, K, epi in SHAPES:
            x, w = uni(M, K), uni(N, K) * 0.02
            nout = N // 2 if epi == "silu" else N
            out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
            e = ops.EPILOGUES[epi]
            variants = {}
            for sk in [int(v) for v in a.sks.split(",")]:
                if (K // 64) < 2 * sk:
                    continue
                sfx = "" if a.sks == "1" else f"/sk{sk}"
                variants["big8" + sfx] = lambda sk=sk: torch.ops.bfly.gemm_with_plan(x, w, out, [4, 0, 0, 0, 256, 256, sk], e, ws)
                variants["big4" + sfx] = lambda sk=sk: torch.ops.bfly.gemm_with_plan(x, w, out, [6, 0, 0, 0, 256, 256, sk], e, ws)
            if a.variants:
                keep = a.variants.split(",")
                variants = {k: v for k, v in variants.items() if k.split("/")[0] in keep}
            if epi == "none" and (not a.variants or "hipblaslt" in a.variants):
                variants["hipblaslt"] = lambda: torch.matmul(x, w.t(), out=out)
            times = {k: [] for k in variants}
            for fn in variants.values():     # warm-up
                fn()
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for k, fn in variants.items():
                    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    st.record()
                    for _ in range(a.iters):
                        fn()
                    en.record()
                    torch.cuda.synchronize()
                    times[k].append(st.elapsed_time(en) / a.iters * 1e3)
            flop = 2.0 * M * N * K
            row = {"shape": name, "M": M, "N": N, "K": K}
            for k, ts in times.items():
                row[k] = {"us_med": round(statistics.median(ts), 1), "us_min": round(min(ts), 1),
                          "TF_med": round(flop / statistics.median(ts) / 1e6, 1)}
            print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
