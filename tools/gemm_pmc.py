#!/usr/bin/env python3
"""Prefill GEMM variants on one Llama-3-70B shape (QKV, 8192 tokens), a few serialized calls
each, for rocprofv3 PMC passes (counters per kernel name: gemm_big8_kernel, plan kind 4;
gemm_big4_kernel, plan kind 6) and
hipBLASLt as the yardstick."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402

assert ops.load_library(), ops._load_error
M, N, K = 8192, 10240, 8192
x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.02).to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
ws = torch.zeros(1 << 20, dtype=torch.float32, device="cuda")
for plan in ([4, 0, 0, 0, 256, 256, 1], [6, 0, 0, 0, 256, 256, 1]):
    for _ in range(4):
        torch.ops.bfly.gemm_with_plan(x, w, out, plan, 0, ws)
        torch.cuda.synchronize()
for _ in range(4):
    torch.matmul(x, w.t(), out=out)
    torch.cuda.synchronize()
print("done")
