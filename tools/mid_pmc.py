#!/usr/bin/env python3
"""Mid-M GEMM plans on two TP-shard shapes, a few serialized calls each, for rocprofv3 PMC
passes (counters per dispatch; rows grouped by plan in call order by tools/mid_pmc_md.py):
tp8 down / QKV at M = 512 and tp4 gate_up at M = 256, each with the 8-wave mid kernel (kind 5)
and the one-wave-per-SIMD mid kernel (kind 7) at the plans the table gives them."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402

assert ops.load_library(), ops._load_error
CASES = [
    ("tp8.down", 512, 8192, 3584, [[5, 4, 4, 0, 128, 128, 1], [7, 4, 6, 0, 128, 128, 1]]),
    ("tp8.qkv", 512, 1280, 8192, [[5, 4, 4, 0, 128, 128, 6], [7, 3, 7, 0, 128, 128, 6]]),
    ("tp4.gate_up", 256, 14336, 8192, [[5, 4, 3, 0, 256, 128, 2], [7, 3, 4, 0, 256, 128, 2]]),
]
ws = torch.zeros(64 << 20, dtype=torch.float32, device="cuda")
log = []
for name, M, N, K, plans in CASES:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.02).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for plan in plans:
        for _ in range(4):
            torch.ops.bfly.gemm_with_plan(x, w, out, plan, 0, ws)
            torch.cuda.synchronize()
        log.append({"shape": name, "M": M, "N": N, "K": K, "plan": plan, "calls": 4})
print(json.dumps(log))
