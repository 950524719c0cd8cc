#!/usr/bin/env python3
"""Run each hot kernel a few times on its production shape (Llama-3-70B, one MI355X) so a
rocprofv3 PMC pass can attribute counters per kernel (tools/profile_counters.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402
from butterfly_amd.ops import reference as ref  # noqa: E402

assert ops.load_library()
dev = "cuda"
torch.manual_seed(0)
bf = torch.bfloat16
R = 3


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device=dev) * scale).to(bf)


# prefill GEMM (gate/up, 8192 tokens) -> big-tile kernel
x = rnd(8192, 8192)
w = rnd(57344, 8192, scale=0.01)
for _ in range(R):
    ops.linear(x, w, epilogue="silu")
# decode GEMMs (B = 64)
xd = rnd(64, 8192)
for _ in range(R):
    ops.linear(xd, w, epilogue="silu")
wd = rnd(8192, 28672, scale=0.01)
hd = rnd(64, 28672)
for _ in range(R):
    ops.linear(hd, wd)
# TP2 replica decode (B = 128): gate/up shard -> decode ring GEMM
w2 = rnd(28672, 8192, scale=0.01)
x2 = rnd(128, 8192)
for _ in range(R):
    ops.linear(x2, w2, epilogue="silu")
del w2
del w, x
torch.cuda.empty_cache()
# decode attention: B=64, ctx 1024, 64 q / 8 kv heads
B, ctx, Hq, Hkv, D, BS = 64, 1024, 64, 8, 128, 32
nb = ctx // BS
kc = rnd(B * nb, Hkv, BS, D)
vc = rnd(B * nb, Hkv, D, BS)
bt = torch.randperm(B * nb, device=dev).to(torch.int32).view(B, nb)
cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
q = rnd(B, Hq, D)
for _ in range(R):
    ops.attn_decode(q, kc, vc, bt, cl, 0.088, ctx)
# prefill attention: 16 x 1024 tokens
T = 16 * 1024
qp, kp, vp = rnd(T, Hq, D), rnd(T, Hkv, D), rnd(T, Hkv, D)
cu = torch.arange(0, T + 1, 1024, dtype=torch.int32, device=dev)
for _ in range(R):
    ops.attn_prefill(qp, kp, vp, cu, 1024, 0.088, True)
# norm / rope
r = rnd(64, 8192)
for _ in range(R):
    ops.rms_norm(xd, rnd(8192), 1e-5, residual=r)
torch.cuda.synchronize()
print("kernel zoo done")
