#!/usr/bin/env python3
"""Mid-M GEMMs under rocprofv3 PMC (round 6): where do the TP-shard projections at M = 512 lose
time? tp8 gate_up (N 7168, K 8192, SiLU) and down (N 8192, K 3584) with the table's mid-M plan,
the 256x256 big4 tile with split-K 4, and torch.matmul (hipBLASLt, yardstick only). Weights
rotate over 3 copies (> the 256 MiB Infinity Cache), as in a decode step that streams every
layer once. Four serialized calls per variant; the log line maps dispatches to variants."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402

assert ops.load_library(), ops._load_error
CASES = [
    ("tp8.gate_up", 512, 7168, 8192, 2, [[7, 4, 3, 0, 128, 256, 2], [6, 0, 0, 0, 256, 256, 4]]),
    ("tp8.down", 512, 8192, 3584, 0, [[7, 4, 6, 0, 128, 128, 1], [6, 0, 0, 0, 256, 256, 4]]),
]
ws = torch.zeros(128 << 20, dtype=torch.float32, device="cuda")
log = []
for name, M, N, K, epi, plans in CASES:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    ws_ = [((torch.rand(N, K, device="cuda") * 2 - 1) * 0.02).to(torch.bfloat16) for _ in range(3)]
    out = torch.empty(M, N // 2 if epi == 2 else N, device="cuda", dtype=torch.bfloat16)
    for plan in plans:
        for i in range(4):
            torch.ops.bfly.gemm_with_plan(x, ws_[i % 3], out, plan, epi, ws)
            torch.cuda.synchronize()
        log.append({"shape": name, "plan": plan, "calls": 4})
    o2 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for i in range(4):
        torch.matmul(x, ws_[i % 3].t(), out=o2)
        torch.cuda.synchronize()
    log.append({"shape": name, "plan": "hipblaslt", "calls": 4})
print(json.dumps(log))
