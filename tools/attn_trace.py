#!/usr/bin/env python3
"""Phase timing inside the persistent prefill attention kernel (BFLY_ATTN_TRACE=1 build path):
wave 0 of every workgroup stamps s_memtime at item start (0), after tile 0's wait (1) and
barrier (2), at the last tile's barrier (3), after the last tile's compute (4) and after the
O stores (5). Prints mean per-item phase lengths in shader-clock ticks.
usage: BFLY_ATTN_TRACE=1 python tools/attn_trace.py [--case 16:1024:64:8] [--noncausal]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from butterfly_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--case", default="16:1024:64:8")
ap.add_argument("--noncausal", action="store_true")
a = ap.parse_args()
ops.load_library()
n, Ls, Hq, Hkv = map(int, a.case.split(":"))
T, D = n * Ls, 128
q = torch.randn(T, Hq, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(T, Hkv, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn(T, Hkv, D, device="cuda", dtype=torch.bfloat16)
cu = torch.arange(0, T + 1, Ls, dtype=torch.int32, device="cuda")
for _ in range(20):
    _, buf = ops.attn_prefill(q, k, v, cu, Ls, 0.088, not a.noncausal, return_lse=True)
torch.cuda.synchronize()
st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
st.record()
_, buf = ops.attn_prefill(q, k, v, cu, Ls, 0.088, not a.noncausal, return_lse=True)
en.record()
torch.cuda.synchronize()
us = st.elapsed_time(en) * 1e3
t = buf.view(-1).view(torch.int64)[: 256 * 32 * 8].view(256, 32, 8).cpu()
valid = t[:, :, 5] > 0
start, w0, b0, bl, ce, end, nt = (t[:, :, i] for i in range(7))
nxt = torch.roll(start, -1, dims=1)
has_next = valid & torch.roll(valid, -1, dims=1)
has_next[:, -1] = False
f = lambda x, m=valid: x[m].double().mean().item()  # noqa: E731
span = (t[:, :, 5].max() - t[:, :, 0][t[:, :, 0] > 0].min()).item()
print(f"case {a.case} causal={not a.noncausal}: kernel {us:.0f} us, traced span {span} ticks "
      f"-> {span / us:.1f} ticks/us")
print(f"  items/WG {valid.sum(1).double().mean():.1f}, tiles/item {f(nt.double()):.1f}")
print(f"  start->tile0 waited   {f(w0 - start):9.0f} ticks")
print(f"  tile0 wait->barrier   {f(b0 - w0):9.0f}")
print(f"  tile0 barrier->last   {f(bl - b0):9.0f}  (per tile {f((bl - b0).double() / (nt - 1).clamp(min=1)):.0f})")
print(f"  last barrier->compute {f(ce - bl):9.0f}")
print(f"  epilogue (stores)     {f(end - ce):9.0f}")
print(f"  end -> next start     {f(nxt - end, has_next):9.0f}")
print(f"  whole item            {f(nxt - start, has_next):9.0f}")
