"""CPU (reference-op) model tests: paged KV decode == full recompute; partition-independent init."""
import torch

from butterfly_amd.config import ModelConfig
from butterfly_amd.engine.batch import make_decode_batch, make_prefill_batch
from butterfly_amd.models import Shard, build_model


def _prefill_logits(model, prompts, bs=32, nblocks=64):
    caches = model.allocate_kv_cache(nblocks, bs)
    slots, tables, nxt = [], [], 0
    for p in prompts:
        nb = (len(p) + 16 + bs - 1) // bs
        blocks = list(range(nxt, nxt + nb))
        nxt += nb
        tables.append(blocks)
        slots.append([blocks[j // bs] * bs + j % bs for j in range(len(p))])
    fb = make_prefill_batch(prompts, slots)
    return model.forward(fb, caches), caches, tables


def _decode(model, caches, tables, tokens, positions, bs=32):
    slots = [tables[i][p // bs] * bs + p % bs for i, p in enumerate(positions)]
    fb = make_decode_batch(tokens, positions, slots, tables, max(len(t) for t in tables), 256)
    return model.forward(fb, caches)


def test_decode_matches_full_recompute():
    torch.manual_seed(0)
    for preset in ("llama-tiny", "mixtral-tiny", "gpt2-tiny"):
        cfg = ModelConfig.from_preset(preset)
        D = cfg.head_dim
        m = build_model(cfg, dtype=torch.float32)
        m.init_random(seed=1)
        prompts = [[5, 17, 99, 3, 8], [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11]]
        logits, caches, tables = _prefill_logits(m, prompts)
        nxt = [int(t) for t in logits.argmax(-1)]
        dec = _decode(m, caches, tables, nxt, [len(p) for p in prompts])
        full, _, _ = _prefill_logits(m, [p + [t] for p, t in zip(prompts, nxt)])
        V = cfg.vocab_size
        assert torch.allclose(dec[:, :V], full[:, :V], atol=1e-4, rtol=1e-4), preset


def test_init_is_partition_independent():
    cfg = ModelConfig.from_preset("llama-tiny")
    full = build_model(cfg, dtype=torch.float32)
    full.init_random(seed=3)
    g = {lp.name: lp.get().clone() for lp in full.logical_params()}
    for tp in (2,):
        for r in range(tp):
            part = build_model(cfg, Shard(tp_rank=r, tp_size=tp), dtype=torch.float32)
            part.init_random(seed=3)
            for lp in part.logical_params():
                ref = g[lp.name]
                if lp.split_dim is not None:
                    ref = ref.narrow(lp.split_dim, lp.offset, lp.length)
                assert torch.equal(lp.get(), ref), lp.name


def test_moe_sparse_reference_matches_dense():
    """The routed expert FFN (reference of the GPU permute/grouped-GEMM path) equals the dense
    gate-scaled formulation on CPU in fp32."""
    import torch
    from butterfly_amd.ops import reference as ref

    g = torch.Generator().manual_seed(0)
    T, E, El, e0, k, H, F = 37, 8, 4, 2, 2, 64, 32
    x = torch.randn(T, H, generator=g)
    wr = torch.randn(E, H, generator=g)
    gates, ids, w = ref.moe_route(x, wr, k)
    gu = torch.randn(El * 2 * F, H, generator=g) / 8
    dn = torch.randn(H, El * F, generator=g) / 8
    sparse = ref.moe_sparse_ffn(x, ids, w, gu, dn, e0, El, F)
    h = ref.linear(x, gu, epilogue="silu")
    ref.moe_gate_scale(h, gates, e0, El)
    dense = ref.linear(h, dn)
    torch.testing.assert_close(sparse, dense, atol=1e-4, rtol=1e-4)


def test_paged_prefill_reference_equals_flash_over_the_whole_prompt():
    """ops.reference.attn_prefill_paged (the oracle of the paged chunked-prefill kernel): a chunk
    at positions [st, st + n) over paged K/V equals the last n rows of causal attention over the
    whole prompt's contiguous K/V."""
    import math

    from butterfly_amd.ops import reference as ref

    torch.manual_seed(5)
    D, BS, Hq, Hkv = 128, 32, 8, 2
    L, st = 150, 97
    k = torch.randn(L, Hkv, D)
    v = torch.randn(L, Hkv, D)
    q = torch.randn(L, Hq, D)
    nb = (L + BS - 1) // BS
    perm = torch.randperm(nb + 3)[:nb]
    kc = torch.zeros(nb + 3, Hkv, BS, D)
    vc = torch.zeros(nb + 3, Hkv, D, BS)
    for t in range(L):
        kc[perm[t // BS], :, t % BS] = k[t]
        vc[perm[t // BS], :, :, t % BS] = v[t]
    i32 = lambda a: torch.tensor(a, dtype=torch.int32)  # noqa: E731
    scale = 1 / math.sqrt(D)
    got = ref.attn_prefill_paged(q[st:], kc, vc, perm.view(1, -1).to(torch.int32), i32([0, L - st]),
                                 i32(list(range(st, L))), L - st, scale)
    want = ref.attn_prefill(q, k, v, i32([0, L]), L, scale, True)[st:]
    torch.testing.assert_close(got, want, atol=1e-5, rtol=1e-5)


def test_moe_decode_fusion_entry_points_fall_back_on_cpu():
    """ops.linear_silu_gate and ops.rms_norm_route (the MoE decode fusions: routing weight in
    the gate/up GEMM epilogue, routing inside the add+RMSNorm) equal their two-op forms on CPU
    tensors, where no fused kernel exists; rms_norm_route without a deferred split-K input
    routes nothing (the caller calls moe_route)."""
    from butterfly_amd import ops
    from butterfly_amd.ops import reference as ref

    g = torch.Generator().manual_seed(7)
    T, H, F, El, E, e0 = 5, 64, 32, 2, 4, 1
    x = torch.randn(T, H, generator=g)
    w = torch.randn(2 * El * F, H, generator=g) * 0.1
    gates = torch.rand(T, E, generator=g)
    got = ops.linear_silu_gate(x, w, gates, e0, El)
    want = ref.linear(x, w, None, "silu")
    ref.moe_gate_scale(want, gates, e0, El)
    torch.testing.assert_close(got, want)
    res = torch.randn(T, H, generator=g)
    nw = torch.rand(H, generator=g) + 0.5
    r1, r2 = res.clone(), res.clone()
    y, route = ops.rms_norm_route(x, nw, 1e-5, r1, torch.randn(E, H, generator=g), 2)
    assert route is None
    torch.testing.assert_close(y, ops.rms_norm(x, nw, 1e-5, residual=r2))
    torch.testing.assert_close(r1, r2)
