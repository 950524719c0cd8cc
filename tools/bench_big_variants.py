#!/usr/bin/env python3
"""A/B the big-tile prefill GEMM variants (BFLY_BIG_VARIANT, csrc/kernels/gemm.hip run_big) on
the Llama-3-70B projection shapes: correctness against torch.matmul, then timing."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402

assert ops.load_library()
variants = (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4,5").split(",")
shapes = [("qkv", 10240, 8192, "none"), ("o", 8192, 8192, "none"), ("gate_up", 57344, 8192, "silu"),
          ("down", 8192, 28672, "none")]
M = int(os.environ.get("BIG_M", "8192"))
ws = torch.zeros(64 << 20, dtype=torch.float32, device="cuda")
for name, N, K, epi in shapes:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    nout = N // 2 if epi == "silu" else N
    out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
    plan = [2, 0, 0, 0, 256, 256, 1]
    ref = None
    for v in variants:
        os.environ["BFLY_BIG_VARIANT"] = v
        f = lambda: torch.ops.bfly.gemm_with_plan(x, w, out, plan, ops.EPILOGUES[epi], ws)  # noqa: E731
        f()
        torch.cuda.synchronize()
        if ref is None:
            ref = out.float().clone()
            if epi == "none":
                want = (x.float() @ w.float().t())
                err = ((ref - want).norm() / want.norm()).item()
            else:
                err = 0.0
        else:
            err = ((out.float() - ref).norm() / ref.norm()).item()
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(10):
            f()
        en.record()
        torch.cuda.synchronize()
        us = st.elapsed_time(en) / 10 * 1e3
        print(json.dumps({"shape": name, "M": M, "variant": v, "us": round(us, 1),
                          "TFLOPs": round(2 * M * N * K / us / 1e6, 1), "rel_err": float(f"{err:.2e}")}), flush=True)
