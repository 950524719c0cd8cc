"""End to end at the BENCH dimensions: the Llama-3-70B, Llama-3-8B and
Mixtral 8x7B presets cut to 2 layers (every projection, the 128k-vocab embedding and LM head at full size),
with the production kernels the benchmark runs:

* prefill of 64 prompts x 128 tokens = 8192 rows through the 256x256 8-phase GEMMs and the
  persistent flash attention, logits against an fp32 PyTorch reference model holding the SAME
  weights (ops.reference_mode: every op of the reference model is the plain torch fp32 op, on the
  same GPU, so no kernel of ours is on the reference side);
* a B = 64 decode step (the bench's batch) through the split-K decode GEMMs, the row-split
  add+RMSNorm and the paged decode attention, eager against the reference, and hipGraph replay
  bitwise against eager.

Mixtral runs the token-routed grouped expert GEMMs in prefill and, in decode, the dense expert
path with routing inside the add+RMSNorm and the routing weight in the gate/up GEMM epilogue.
Routing is a discrete choice: a token whose top-2 experts nearly tie can pick another expert in
bf16 than in fp32, so for MoE presets 90 % of the rows must match individually (a flip changes
one token's row, not the others), each within 2.5x the dense bound.
"""
import dataclasses

import pytest
import torch

from butterfly_amd import ops
from butterfly_amd.config import ModelConfig
from butterfly_amd.engine.batch import make_decode_batch, make_prefill_batch
from butterfly_amd.models import build_model

pytestmark = pytest.mark.gpu

BS = 32


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm()).item()


def _check(a, b, tol, moe):
    if not moe:
        rel = _rel(a, b)
        assert rel < tol, f"logits rel err {rel:.3e}"
        return
    # per-row bf16 noise through the expert GEMMs is ~2 % here (median row error 2.2e-2 in the
    # prefill of the first run), so the per-row bound is 2.5x the dense presets' whole-matrix bound
    a, b = a.float(), b.float()
    rows = (a - b).norm(dim=-1) / b.norm(dim=-1)
    ok = (rows < 2.5 * tol).float().mean().item()
    print(f"moe logits: median row rel err {rows.median().item():.3e}, {ok:.0%} within {2.5 * tol}")
    assert ok >= 0.9, f"only {ok:.0%} of rows within {2.5 * tol} (median {rows.median().item():.3e})"


def _models(preset):
    cfg = dataclasses.replace(ModelConfig.from_preset(preset), num_layers=2)
    g = build_model(cfg, device="cuda", dtype=torch.bfloat16)
    g.init_random(seed=5)
    with ops.reference_mode():
        r = build_model(cfg, device="cuda", dtype=torch.float32)
    for k, v in g.p.items():
        r.p[k].copy_(v.float())
    return cfg, g, r


@pytest.mark.parametrize("preset", ["llama3-8b", "llama3-70b", "mixtral-8x7b"])
def test_bench_dims_prefill_decode_and_graph(preset):
    cfg, g, r = _models(preset)
    V = cfg.vocab_size
    B, P = 64, 128
    gen = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, V, (P,), generator=gen).tolist() for _ in range(B)]
    nb = (P + 1 + BS - 1) // BS + 1
    tables = [list(range(i * nb, (i + 1) * nb)) for i in range(B)]
    slots = [[tables[i][j // BS] * BS + j % BS for j in range(P)] for i in range(B)]
    kg = g.allocate_kv_cache(B * nb + 1, BS)
    with ops.reference_mode():
        kr = r.allocate_kv_cache(B * nb + 1, BS)

    fb = make_prefill_batch(prompts, slots).to("cuda")
    assert fb.num_tokens == 8192
    lg = g.forward(fb, kg)
    with ops.reference_mode():
        lr = r.forward(fb, kr)
    torch.cuda.synchronize()
    assert lg.shape[0] == B
    _check(lg[:, :V], lr[:, :V], 2e-2, cfg.is_moe)

    toks = [int(t) for t in lr[:, :V].argmax(-1)]
    pos = [P] * B
    sl = [tables[i][P // BS] * BS + P % BS for i in range(B)]
    db = make_decode_batch(toks, pos, sl, tables, nb, nb * BS).to("cuda")
    kg_snapshot = [(k.clone(), v.clone()) for k, v in kg]
    dg = g.forward(db, kg)
    kv_eager = [(k.clone(), v.clone()) for k, v in kg]
    with ops.reference_mode():
        dr = r.forward(db, kr)
    torch.cuda.synchronize()
    _check(dg[:, :V], dr[:, :V], 3e-2, cfg.is_moe)

    # the decode step over the K-tile-blocked copies the engine makes by default
    # (BFLY_PACKED_KINDS; what an engine with HBM to spare runs): they run the row-major plans,
    # so bitwise the eager logits and cache writes (a kind with its own packed plan in
    # gemm.hip kPackedTuned, e.g. the 70B O projection, sums its split-K in another order)
    for (k, v), (k0, v0) in zip(kg, kg_snapshot):
        k.copy_(k0)
        v.copy_(v0)
    dg_eager = dg.clone()
    g.pack_decode_weights(kinds=["gu_w", "moe_gu_w", "qkv_w"])
    assert g.packed
    dp = g.forward(db, kg)
    torch.cuda.synchronize()
    assert torch.equal(dp, dg_eager), "decode over the packed gate/up weights differs"
    for (k, v), (k1, v1) in zip(kg, kv_eager):
        assert torch.equal(k, k1) and torch.equal(v, v1)

    # hipGraph replay of the same decode step: bitwise the eager logits and cache writes
    for (k, v), (k0, v0) in zip(kg, kg_snapshot):
        k.copy_(k0)
        v.copy_(v0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            g.forward(db, kg)
    torch.cuda.current_stream().wait_stream(s)
    for (k, v), (k0, v0) in zip(kg, kg_snapshot):
        k.copy_(k0)
        v.copy_(v0)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = g.forward(db, kg)
    for (k, v), (k0, v0) in zip(kg, kg_snapshot):
        k.copy_(k0)
        v.copy_(v0)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, dg), "graph replay differs from eager"
    for (k, v), (k1, v1) in zip(kg, kv_eager):
        assert torch.equal(k, k1) and torch.equal(v, v1)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, dg), "second replay differs"
    for (k, v), (k1, v1) in zip(kg, kv_eager):
        assert torch.equal(k, k1) and torch.equal(v, v1)
