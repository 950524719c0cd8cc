#!/usr/bin/env python3
"""Mid-M GEMM plans on two TP-shard shapes, a few serialized calls each, for rocprofv3 PMC
passes (counters per dispatch; rows grouped by plan in call order by tools/mid_pmc_md.py):
tp8 down at M = 512 (N 8192, K 3584) and tp4 gate_up at M = 256 (N 14336, K 8192), each with
the mid8 kernel (kind 5), the 4-wave tile kernel (kind 1) and the 8-phase big tile (kind 4)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402

assert ops.load_library(), ops._load_error
CASES = [
    ("tp8.down", 512, 8192, 3584, [[5, 3, 0, 0, 256, 128, 2], [5, 4, 0, 0, 128, 128, 1], [1, 4, 0, 2, 128, 128, 1],
                                   [4, 0, 0, 0, 256, 256, 4]]),
    ("tp4.gate_up", 256, 14336, 8192, [[5, 3, 0, 0, 256, 128, 2], [5, 3, 0, 0, 256, 128, 1], [1, 2, 0, 2, 128, 128, 2],
                                       [4, 0, 0, 0, 256, 256, 4]]),
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
