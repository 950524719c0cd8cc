"""Numerics of every HIP kernel against the plain-PyTorch fp32 reference (ops/reference.py).

Random normal (asymmetric) operands throughout: a symmetric or identity operand hides a
transposed C-write (cdna_hip_programming.md §3, "Always A=I-check with ASYMMETRIC B").
"""
import math
import os

import pytest
import torch

from butterfly_amd import ops
from butterfly_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _kernels_loaded():
    # GPU tests must run the HIP kernels: fail loudly if the library is missing
    assert ops.load_library(), "butterfly_amd/_C.so not built or failed to load"


def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).to(DEV)


def _close(a, b, atol, rtol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad}/{a.numel()} mismatches, max err {err.max().item():.4g}"


def test_native_library_loaded():
    assert ops.native_available(), ops._load_error


@pytest.mark.parametrize("rows,dim", [(1, 768), (7, 4096), (64, 8192), (3, 16384)])
@pytest.mark.parametrize("with_res", [False, True])
def test_rms_norm(rows, dim, with_res):
    x = _bf(rows, dim, seed=1)
    w = _bf(dim, seed=2)
    res = _bf(rows, dim, seed=3) if with_res else None
    res_ref = res.clone() if with_res else None
    y = ops.rms_norm(x, w, 1e-5, residual=res)
    y_ref = ref.rms_norm(x, w, 1e-5, residual=res_ref)
    _close(y, y_ref, 2e-2, 2e-2)
    if with_res:
        _close(res, res_ref, 0, 0)


@pytest.mark.parametrize("with_res", [False, True])
def test_layer_norm(with_res):
    x = _bf(9, 768, seed=4)
    w, b = _bf(768, seed=5), _bf(768, seed=6)
    res = _bf(9, 768, seed=7) if with_res else None
    res_ref = res.clone() if with_res else None
    _close(ops.layer_norm(x, w, b, 1e-5, residual=res), ref.layer_norm(x, w, b, 1e-5, residual=res_ref), 3e-2, 2e-2)


def test_rope_kv_and_cache():
    T, Hq, Hkv, D, BS, nblk = 37, 8, 2, 128, 32, 6
    qkv = _bf(T, (Hq + 2 * Hkv) * D, seed=8)
    pos = torch.randint(0, 500, (T,), dtype=torch.int32, device=DEV)
    cos, sin = ref.rope_tables(D, 1024, 500000.0, device=DEV)
    slots = torch.randperm(nblk * BS, device=DEV)[:T].to(torch.int32)
    slots[3] = -1
    kc = torch.zeros(nblk, Hkv, BS, D, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros(nblk, Hkv, D, BS, dtype=torch.bfloat16, device=DEV)
    q2, kc2, vc2 = qkv.clone(), kc.clone(), vc.clone()
    ops.rope_kv(qkv, pos, cos, sin, Hq, Hkv, slots, kc, vc)
    ref.rope_kv(q2, pos, cos, sin, Hq, Hkv, slots, kc2, vc2)
    _close(qkv, q2, 1e-2, 1e-2)
    _close(kc, kc2, 1e-2, 1e-2)
    _close(vc, vc2, 0, 0)


@pytest.mark.parametrize("interleave", [0, 16])
def test_silu_mul(interleave):
    gu = _bf(13, 2 * 1024, seed=9)
    _close(ops.silu_mul(gu, interleave=interleave), ref.silu_mul(gu, interleave=interleave), 1e-2, 1e-2)


def test_gelu_add():
    x, y = _bf(5, 3072, seed=10), _bf(5, 3072, seed=11)
    _close(ops.gelu(x), ref.gelu(x), 1e-2, 1e-2)
    _close(ops.add(x, y), ref.add(x, y), 1e-2, 1e-2)


def test_embed_vocab_parallel():
    table = _bf(1000, 512, seed=12)
    ids = torch.tensor([0, 5, 999, 1000, 1500, 2999, 1234], dtype=torch.int32, device=DEV)
    _close(ops.embed(ids, table, vstart=1000), ref.embed(ids, table, vstart=1000), 0, 0)


@pytest.mark.parametrize("V", [1000, 32000, 128256])
def test_sample_greedy(V):
    logits = _bf(6, V, seed=13)
    ids, scores = ops.sample(logits)
    exp = logits.float().argmax(-1)
    assert torch.equal(ids.long().cpu(), exp.cpu())
    _close(scores, logits.float().max(-1).values, 1e-3, 1e-3)


def test_sample_gumbel_matches_reference():
    V = 4096
    logits = _bf(3, V, seed=14)
    temps = torch.tensor([0.0, 0.7, 1.3], device=DEV)
    seeds = torch.tensor([1, 42, 12345], dtype=torch.int64, device=DEV)
    ids, _ = ops.sample(logits, temps, seeds, vstart=0)
    ids_ref, _ = ref.sample(logits.cpu(), temps.cpu(), seeds.cpu(), vstart=0)
    assert ids.cpu().tolist() == ids_ref.tolist()


def test_sample_topk_topp_on_device():
    """Filtered sampling on the GPU: the radix-select thresholds (tkp_* kernels) equal the
    tie-aware exact ones on a 128k vocabulary with high-entropy rows (nuclei of thousands of
    tokens), equal the CPU reference's, and the thresholded Gumbel kernel then picks exactly
    what the fp32 reference picks."""
    from butterfly_amd.engine.sampler import Sampler, SamplingParams
    from tests.test_sampler import value_threshold

    V = 128256
    params = [SamplingParams(temperature=0.8, top_k=20), SamplingParams(temperature=1.0, top_p=0.9),
              SamplingParams(temperature=0.6, top_k=5000, top_p=0.95), SamplingParams(temperature=0.0),
              SamplingParams(temperature=1.2, top_p=0.3), SamplingParams(temperature=1.0, top_k=1)]
    logits = _bf(len(params), V, scale=0.6, seed=17)
    temps = torch.tensor([p.temperature for p in params], device=DEV)
    seeds = torch.arange(3, 3 + len(params), dtype=torch.int64, device=DEV)
    smp = Sampler(None, V, 0, 1)
    thr = smp.thresholds(logits, temps, params)
    thr_cpu = Sampler(None, V, 0, 1).thresholds(logits.cpu(), temps.cpu(), params)
    for r, p in enumerate(params):
        if p.temperature <= 0:
            assert float(thr[r]) == float("-inf")
            continue
        want = value_threshold(logits[r].cpu(), p.temperature, p.top_k, p.top_p)
        assert float(thr[r]) == want, (r, float(thr[r]), want)
        assert float(thr_cpu[r]) == want
    ids, _ = ops.sample(logits, temps, seeds, vstart=0, thresh=thr)
    ids_ref, _ = ref.sample(logits.cpu(), temps.cpu(), seeds.cpu(), vstart=0, thresh=thr.cpu())
    assert ids.cpu().tolist() == ids_ref.tolist()
    got = smp.sample(logits, temps, seeds, params)
    assert torch.equal(got.cpu(), ids.cpu())
    assert int(ids[3]) == int(logits[3].float().argmax())
    assert int(ids[5]) == int(logits[5].float().argmax())


def test_topkp_all_negative_logits_low_temperature():
    """Rows whose scaled logits are all far below zero: the radix select must start from the
    true row maximum (not +0.0), or exp(s - 0) underflows, Z becomes 0 and top-p silently
    keeps every token. GPU thresholds must equal the CPU reference's and the exact ones."""
    from butterfly_amd.engine.sampler import Sampler, SamplingParams
    from tests.test_sampler import value_threshold

    V = 32000
    params = [SamplingParams(temperature=0.05, top_p=0.9), SamplingParams(temperature=0.1, top_k=7, top_p=0.5),
              SamplingParams(temperature=0.02, top_k=3)]
    logits = (_bf(len(params), V, scale=0.5, seed=23).float() - 30.0).to(torch.bfloat16)
    temps = torch.tensor([p.temperature for p in params], device=DEV)
    thr = Sampler(None, V, 0, 1).thresholds(logits, temps, params)
    thr_cpu = Sampler(None, V, 0, 1).thresholds(logits.cpu(), temps.cpu(), params)
    for r, p in enumerate(params):
        want = value_threshold(logits[r].cpu(), p.temperature, p.top_k, p.top_p)
        assert float(thr[r]) == want, (r, float(thr[r]), want)
        assert float(thr_cpu[r]) == want
        assert want > float("-inf")   # the filter is active: not every token qualifies


@pytest.mark.parametrize("tp", [2, 4])
def test_sample_filtered_vocab_parallel_on_device(tp):
    """Vocab-parallel shards on the GPU (loopback TP ranks sharing the device): histograms are
    summed across shards, shards left without a candidate (top_k = 1, tiny top_p) score -inf,
    and the merged ids equal the single-shard ids."""
    from butterfly_amd.engine.sampler import Sampler, SamplingParams
    from butterfly_amd.parallel.fake import FakeWorld
    from butterfly_amd.parallel.mesh import Mesh

    V = 32768
    params = [SamplingParams(temperature=1.0, top_k=1), SamplingParams(temperature=0.8, top_p=0.02),
              SamplingParams(temperature=1.1, top_k=3000, top_p=0.9), SamplingParams(temperature=0.0)]
    logits = _bf(len(params), V, scale=2.0, seed=23)
    temps = torch.tensor([p.temperature for p in params], device=DEV)
    seeds = torch.arange(5, 5 + len(params), dtype=torch.int64, device=DEV)
    one = Sampler(None, V, 0, 1).sample(logits, temps, seeds, params, check_finite=True)
    assert int(one[0]) == int(logits[0].float().argmax())
    world = FakeWorld(Mesh(tp=tp))

    def body(rank, comm):
        Vl = V // tp
        return Sampler(comm, V, rank * Vl, tp).sample(logits[:, rank * Vl:(rank + 1) * Vl].contiguous(), temps,
                                                      seeds, params, check_finite=True)

    for ids in world.run(body):
        assert ids.cpu().tolist() == one.cpu().tolist()


GEMM_SHAPES = [
    (1, 256, 1024), (5, 1280, 8192), (16, 4096, 4096), (33, 512, 768), (64, 2048, 1024),
    (65, 256, 512), (128, 1024, 2048), (300, 384, 640), (1024, 1024, 1024), (7, 16128, 8192),
]


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
def test_gemm(M, N, K):
    x = _bf(M, K, seed=15)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=16)
    y = ops.linear(x, w)
    _close(y, ref.linear(x, w), 2e-2, 2e-2)


@pytest.mark.parametrize("M", [1, 16, 40, 64, 200])
def test_gemm_bias_and_silu(M):
    K, N = 1024, 512
    x = _bf(M, K, seed=17)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=18)
    b = _bf(N, seed=19)
    _close(ops.linear(x, w, bias=b), ref.linear(x, w, bias=b), 2e-2, 2e-2)
    _close(ops.linear(x, w, epilogue="silu"), ref.linear(x, w, epilogue="silu"), 2e-2, 2e-2)


@pytest.mark.parametrize("Hq,Hkv", [(8, 2), (4, 4), (64, 8)])
def test_attn_prefill_varlen_causal(Hq, Hkv):
    D = 128
    lens = [1, 37, 128, 200]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = sum(lens)
    qkv = _bf(T, (Hq + 2 * Hkv) * D, seed=20)
    q = qkv[:, : Hq * D].view(T, Hq, D)
    k = qkv[:, Hq * D: (Hq + Hkv) * D].view(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:].view(T, Hkv, D)
    scale = 1.0 / math.sqrt(D)
    o = ops.attn_prefill(q, k, v, cu, max(lens), scale, True)
    _close(o, ref.attn_prefill(q, k, v, cu, max(lens), scale, True), 2e-2, 2e-2)


def test_attn_prefill_non_causal():
    D, Hq, Hkv = 128, 4, 2
    lens = [70, 130]
    cu = torch.tensor([0, 70, 200], dtype=torch.int32, device=DEV)
    q, k, v = _bf(200, Hq, D, seed=21), _bf(200, Hkv, D, seed=22), _bf(200, Hkv, D, seed=23)
    o = ops.attn_prefill(q, k, v, cu, 130, 0.088, False)
    _close(o, ref.attn_prefill(q, k, v, cu, 130, 0.088, False), 2e-2, 2e-2)


@pytest.mark.parametrize("part_tokens", [0, 128, 256, 4096])
@pytest.mark.parametrize("Hq,Hkv", [(16, 2), (8, 8), (64, 8)])
def test_attn_decode_paged(part_tokens, Hq, Hkv):
    D, BS = 128, 32
    lens = [1, 31, 32, 100, 700]
    B = len(lens)
    max_blocks = (max(lens) + BS - 1) // BS
    nblk = B * max_blocks + 3
    kc = _bf(nblk, Hkv, BS, D, seed=24)
    vc = _bf(nblk, Hkv, D, BS, seed=25)
    perm = torch.randperm(nblk)[: B * max_blocks].view(B, max_blocks).to(torch.int32).to(DEV)
    ctx = torch.tensor(lens, dtype=torch.int32, device=DEV)
    q = _bf(B, Hq, D, seed=26)
    scale = 1.0 / math.sqrt(D)
    want = ref.attn_decode(q, kc, vc, perm, ctx, scale)
    o = ops.attn_decode(q, kc, vc, perm, ctx, scale, max(lens), part_tokens)
    _close(o, want, 2e-2, 2e-2)


def _paged_chunk_case(Hq, Hkv, kv_dtype, seed=40, pre=(0, 40, 95, 700, 31), chunk=(37, 1, 50, 16, 129)):
    """Sequences with (cached prefix, chunk) lengths, their pages scattered over a pool with
    holes (random permutation, unused blocks in between), queries as a fused-QKV row view."""
    D, BS = 128, 32
    S = len(pre)
    maxb = max((p + c + BS - 1) // BS for p, c in zip(pre, chunk))
    nblk = S * maxb + 7
    kc = _bf(nblk, Hkv, BS, D, seed=seed)
    vc = _bf(nblk, Hkv, D, BS, seed=seed + 1)
    if kv_dtype == "fp8":
        kc, vc = kc.to(torch.float8_e4m3fn), vc.to(torch.float8_e4m3fn)
    g = torch.Generator().manual_seed(seed + 2)
    tables = torch.randperm(nblk, generator=g)[: S * maxb].view(S, maxb).to(torch.int32).to(DEV)
    T = sum(chunk)
    qkv = _bf(T, (Hq + 2 * Hkv) * D, seed=seed + 3)
    q = qkv[:, : Hq * D].view(T, Hq, D)
    cu = [0]
    pos = []
    for p, c in zip(pre, chunk):
        cu.append(cu[-1] + c)
        pos.extend(range(p, p + c))
    i32 = lambda a: torch.tensor(a, dtype=torch.int32, device=DEV)  # noqa: E731
    return q, kc, vc, tables, i32(cu), i32(pos), max(chunk)


@pytest.mark.parametrize("Hq,Hkv", [(64, 8), (32, 8), (8, 2), (8, 8), (12, 4), (16, 16)])
@pytest.mark.parametrize("kv_dtype", ["bf16", "fp8"])
def test_attn_prefill_paged_vs_fp32(Hq, Hkv, kv_dtype):
    """Chunked prefill over the paged cache (attention_paged.hip): prefixes of 0 .. 700 cached
    tokens, chunks of 1 .. 129 tokens (ragged 16-token blocks), pages with holes, bf16 and FP8
    pages, GQA groups of 8 / 4 / 4 / 1 — against the fp32 reference over the same pages."""
    q, kc, vc, tables, cu, pos, mq = _paged_chunk_case(Hq, Hkv, kv_dtype)
    scale = 1.0 / math.sqrt(128)
    o = ops.attn_prefill_paged(q, kc, vc, tables, cu, pos, mq, scale)
    want = ref.attn_prefill_paged(q.cpu(), kc.cpu(), vc.cpu(), tables.cpu(), cu.cpu(), pos.cpu(), mq, scale)
    _close(o, want, 2e-2, 2e-2)


@pytest.mark.parametrize("Hq,Hkv", [(64, 8), (32, 8)])
@pytest.mark.parametrize("kv_dtype", ["bf16", "fp8"])
def test_attn_prefill_paged_single_sequence(Hq, Hkv, kv_dtype):
    """One sequence's chunk (the launcher's register-kernel path) over a 700-token prefix."""
    q, kc, vc, tables, cu, pos, mq = _paged_chunk_case(Hq, Hkv, kv_dtype, seed=60, pre=(700,), chunk=(129,))
    scale = 1.0 / math.sqrt(128)
    o = ops.attn_prefill_paged(q, kc, vc, tables, cu, pos, mq, scale)
    want = ref.attn_prefill_paged(q.cpu(), kc.cpu(), vc.cpu(), tables.cpu(), cu.cpu(), pos.cpu(), mq, scale)
    _close(o, want, 2e-2, 2e-2)


def test_attn_decode_strided_q():
    # q as a view into a fused QKV row (row stride > Hq*D), as the model passes it
    D, BS, Hq, Hkv, B = 128, 32, 8, 1, 3
    qkv = _bf(B, (Hq + 2 * Hkv) * D, seed=27)
    q = qkv[:, : Hq * D].view(B, Hq, D)
    kc, vc = _bf(8, Hkv, BS, D, seed=28), _bf(8, Hkv, D, BS, seed=29)
    bt = torch.arange(8, dtype=torch.int32, device=DEV).view(1, 8).repeat(B, 1)
    ctx = torch.tensor([5, 64, 250], dtype=torch.int32, device=DEV)
    o = ops.attn_decode(q, kc, vc, bt, ctx, 0.1, 256)
    _close(o, ref.attn_decode(q, kc, vc, bt, ctx, 0.1), 2e-2, 2e-2)


def test_init_hash_matches_reference_and_is_partition_independent():
    full = torch.empty(96, 256, dtype=torch.bfloat16, device=DEV)
    ops.init_hash_(full, 0, 0, 256, 1234, 0.1)
    cpu = torch.empty(96, 256, dtype=torch.bfloat16)
    ref.init_hash(cpu, 0, 0, 256, 1234, 0.1)
    _close(full, cpu, 1e-3, 1e-2)
    part = torch.empty(32, 128, dtype=torch.bfloat16, device=DEV)
    ops.init_hash_(part, 40, 64, 256, 1234, 0.1)
    assert torch.equal(part.cpu(), full[40:72, 64:192].cpu())


def test_moe_route_and_gate_scale():
    T, H, E, K = 37, 512, 8, 2
    x, wr = _bf(T, H, seed=30), _bf(E, H, scale=0.05, seed=31)
    g, ids, w = ops.moe_route(x, wr, K)
    g2, ids2, w2 = ref.moe_route(x, wr, K)
    _close(g, g2, 1e-3, 1e-2)
    h = _bf(T, 3 * 64, seed=32)
    h2 = h.clone()
    ops.moe_gate_scale_(h, g, 2, 3)
    ref.moe_gate_scale(h2, g2, 2, 3)
    _close(h, h2, 1e-2, 1e-2)


@pytest.mark.parametrize("T,dim,sk,k,E", [(64, 4096, 4, 2, 8), (37, 4096, 1, 2, 8), (5, 8192, 3, 1, 8), (130, 1024, 2, 3, 8),
                                         (40, 256, 2, 2, 4)])
def test_rms_norm_route_equals_norm_then_route(T, dim, sk, k, E):
    """ops.rms_norm_route (the add+RMSNorm over split-K slabs that also routes its rows for a
    MoE layer): the normalised rows and the residual are bit-identical to rms_norm_partial, and
    gates / top-k match moe_route on those rows (same softmax / top-k code; the router dot
    products sum in a different order, so gates agree to f32 rounding and the chosen experts
    are the same unless two probabilities tie to within it)."""
    slabs = (torch.randn(sk, T, dim, generator=torch.Generator().manual_seed(80)) * 0.5).to(DEV)
    res0 = _bf(T, dim, seed=81)
    w = (1.0 + 0.1 * _bf(dim, seed=82).float()).to(torch.bfloat16)
    wr = _bf(E, dim, scale=0.05, seed=83)
    part = ops.Partial(slabs, torch.empty(T, dim, dtype=torch.bfloat16, device=DEV))
    res_a = res0.clone()
    y, route = ops.rms_norm_route(part, w, 1e-5, res_a, wr, k)
    assert route is not None
    gates, ids, tw = route
    res_b = res0.clone()
    y_ref = ops.rms_norm(part, w, 1e-5, residual=res_b)
    assert torch.equal(y, y_ref) and torch.equal(res_a, res_b)
    g2, ids2, tw2 = ops.moe_route(y_ref, wr, k)
    _close(gates, g2, 1e-5, 1e-4)
    _close(tw, tw2, 1e-5, 1e-4)
    p = torch.softmax((y_ref.float() @ wr.float().t()), dim=-1).cpu()
    srt = p.sort(dim=-1, descending=True).values
    clear = (srt[:, k - 1] - srt[:, k]) > 1e-4          # no near-tie at the top-k boundary
    assert clear.sum() >= T // 2
    assert torch.equal(ids.cpu()[clear].sort(dim=-1).values, ids2.cpu()[clear].sort(dim=-1).values)


@pytest.mark.parametrize("M,N,K,mode", [(64, 57344, 8192, "silu"), (64, 28672, 4096, "rowscale"),
                                         (48, 28672, 4096, "silu"), (64, 2 * 2 * 14336, 4096, "gate"),
                                         (16, 28672, 4096, "silu"), (200, 28672, 4096, "silu"),
                                         (64, 10240, 8192, "defer"), (64, 8192, 8192, "defer"),
                                         (64, 8192, 28672, "defer"), (64, 4096, 114688, "defer"),
                                         (64, 4096, 14336, "none"), (1, 57344, 8192, "silu"),
                                         (3, 28672, 4096, "rowscale"), (1, 4096, 14336, "none"),
                                         (1, 10240, 8192, "defer"), (8, 8192, 28672, "defer"),
                                         (24, 8192, 8192, "defer"), (128, 8192, 8192, "defer"),
                                         (256, 8192, 8192, "defer"), (128, 8192, 4096, "none"),
                                         (256, 28672, 8192, "silu"), (256, 5120, 8192, "defer"),
                                         (600, 28672, 4096, "silu"), (64, 4096, 4096, "keep")])
def test_packed_decode_gemm_is_bitwise_the_row_major_one(M, N, K, mode):
    """The decode GEMM over the K-tile-blocked copy of a weight (ops.pack_w256, gemm.hip
    launch_gemm_packed) runs the plan the row-major weight would run with the same arithmetic
    order: bitwise the same output, for the SwiGLU epilogue, with a row-split RMSNorm row scale
    and with the MoE gate, down to the 16 / 32-row tiles of the B = 1-32 latency buckets and up
    to the mid-M kernels (plan kinds 5 / 7, M = 128-256, split-K slabs included); shapes whose
    plan has no packed form (M = 600: the 256 x 256 prefill tile) report so and ops.linear
    falls back to the row-major weight."""
    x, w = _bf(M, K, seed=90), _bf(N, K, scale=0.02, seed=91)
    wp = ops.pack_w256(w)
    if mode == "gate":
        E, El = 8, 2
        gates = torch.rand(M, E, generator=torch.Generator().manual_seed(92)).to(DEV)
        got = ops.linear_silu_gate(x, w, gates, 3, El, packed=wp)
        want = ops.linear_silu_gate(x, w, gates, 3, El)
        assert torch.equal(got, want)
        out = torch.empty_like(got)
        assert torch.ops.bfly.gemm_packed(x, wp, out, 3, None, 0.0, gates, 3, El) > 0
        return
    if mode == "keep":
        # a shape the packed table keeps on the row-major weight: no packed plan, same result
        assert torch.ops.bfly.gemm_packed_check(M, N, K, 0) != 0
        assert torch.equal(ops.linear(x, w, packed=wp), ops.linear(x, w))
        return
    if mode in ("defer", "none"):
        # split-K plans over the packed copy: the slabs (deferred, as for the QKV / O / down
        # projections the consumer reduces) and the reduced output are bitwise the row-major ones
        d = mode == "defer"
        own = {(64, 8192, 8192): [1, 3, 0, 2, 64, 128, 4]}.get((M, N, K))
        if own is not None:
            # a packed-table plan (gemm.hip kPackedTuned): bitwise the row-major weight on that plan
            got = ops.linear(x, w, packed=wp).clone()   # both through the plan's own split-K reduce
            want = torch.empty_like(got)
            torch.ops.bfly.gemm_with_plan(x, w, want, own, 0, torch.zeros(16 << 20, dtype=torch.float32, device=DEV))
            assert torch.equal(got, want)
            _close(got, x.float() @ w.float().t(), 2e-2, 2e-2)
            return
        got = ops.linear(x, w, defer=d, packed=wp)      # slabs live in the shared GEMM workspace:
        got_slabs = got.slabs.clone() if isinstance(got, ops.Partial) else None   # copy before the next GEMM
        got = ops.materialize(got).clone()
        want = ops.linear(x, w, defer=d)
        if d:
            assert (got_slabs is None) == (not isinstance(want, ops.Partial))
            if got_slabs is not None:
                assert torch.equal(got_slabs, want.slabs)
        want = ops.materialize(want)
        assert torch.equal(got, want)
        _close(got, x.float() @ w.float().t(), 2e-2, 2e-2)
        assert torch.ops.bfly.gemm_packed_check(M, N, K, 0) == 0
        return
    if mode == "rowscale":
        res = _bf(M, K, seed=93)
        nw = (1.0 + 0.1 * _bf(K, seed=94).float()).to(torch.bfloat16)
        xin = ops.rms_norm(x, nw, 1e-5, residual=res.clone(), rows=True)
    else:
        xin = x
    got = ops.linear(xin, w, epilogue="silu", packed=wp)
    want = ops.linear(xin, w, epilogue="silu")
    assert torch.equal(got, want)
    out = torch.empty_like(got)
    applies = torch.ops.bfly.gemm_packed(x, wp, out, ops.EPILOGUES["silu"]) > 0
    assert applies == (M <= 256), (M, applies)


@pytest.mark.parametrize("M,El,e0,E,H,F", [(64, 8, 0, 8, 512, 256), (37, 3, 2, 8, 256, 128), (130, 2, 0, 4, 1024, 512),
                                           (16, 4, 4, 8, 512, 64), (64, 1, 3, 8, 4096, 14336)])
def test_gate_scaled_silu_epilogue(M, El, e0, E, H, F):
    """ops.linear_silu_gate (the routing weight applied in the tile kernel's SwiGLU epilogue,
    EPI_SILU_GATE) is bit-identical to the same plan's SiLU GEMM followed by moe_gate_scale,
    and matches the fp32 reference; zero gates (unselected experts) give exact zeros. The last
    case is one Mixtral 8x7B expert at the decode batch."""
    x, w = _bf(M, H, seed=70), _bf(2 * El * F, H, scale=0.05, seed=71)
    g = torch.Generator(device="cpu").manual_seed(72)
    gates = torch.rand(M, E, generator=g)
    gates[torch.rand(M, E, generator=g) < 0.5] = 0.0
    gates = gates.to(DEV)
    N, K = w.shape[0], H
    got = ops.linear_silu_gate(x, w, gates, e0, El)
    p = ops.gemm_plan(M, N, K)
    if p["kind"] == "tile" and p["splitk"] == 1:
        plan = [1, p["mt"], p["nt"], p["wk"], p["bm"], p["bn"], 1]
    else:
        bm = 16 if M <= 16 else 32 if M <= 32 else 64 if M <= 64 else 128
        plan = [1, 3, 0, 1 if bm <= 32 else 2, bm, 128, 1]
    base = torch.empty(M, N // 2, dtype=torch.bfloat16, device=DEV)
    torch.ops.bfly.gemm_with_plan(x, w, base, plan, ops.EPILOGUES["silu"], None)
    ops.moe_gate_scale_(base, gates, e0, El)
    assert torch.equal(got, base)
    want = ref.linear(x.cpu(), w.cpu(), None, "silu")
    ref.moe_gate_scale(want, gates.cpu(), e0, El)
    _close(got, want, 2e-2, 2e-2)
    cols = torch.arange(N // 2) // F + e0
    off = (gates.cpu()[:, cols] == 0)
    assert (got.cpu()[off] == 0).all()


@pytest.mark.parametrize("M,N,K", [(600, 512, 1024), (256, 768, 192), (77, 256, 128), (1000, 1280, 4096),
                                   (300, 512, 256), (520, 512, 128)])
@pytest.mark.parametrize("kind", [4, 6])
@pytest.mark.parametrize("epi", ["none", "bias", "silu"])
def test_gemm_big_tile(M, N, K, epi, kind):
    """256x256 prefill kernels (plan kind 4: 8-phase, 8 waves; kind 6: one wave per SIMD):
    ragged M, the minimum of two 64-deep K-tiles per split, uneven split-K, all epilogues,
    asymmetric operands."""
    x = _bf(M, K, seed=60)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=61)
    b = _bf(N, seed=62) if epi == "bias" else None
    nout = N // 2 if epi == "silu" else N
    want = ref.linear(x, w, b, "silu" if epi == "silu" else "none")
    for sk in (1, 2, 3):
        if K // 64 < 2 * sk:
            continue
        out = torch.empty(M, nout, dtype=torch.bfloat16, device=DEV)
        ws = torch.zeros(sk * M * N + 16384, dtype=torch.float32, device=DEV)
        torch.ops.bfly.gemm_with_plan(x, w, out, [kind, 0, 0, 0, 256, 256, sk], ops.EPILOGUES[epi], ws, b)
        _close(out, want, 2e-2, 2e-2)


@pytest.mark.parametrize("kind", [4, 6])
@pytest.mark.parametrize("M,N,K,epi,sk", [(4096, 4096, 8192, "none", 1),      # 256-tile grid, K 8192
                                          (8192, 2560, 8192, "silu", 1),      # 70B prefill shapes
                                          (520, 7168, 8192, "silu", 4),       # tp8 gate_up at M 512+
                                          (512, 1280, 8192, "none", 8)])      # tp8 QKV, deep split
def test_gemm_big_tile_production(M, N, K, epi, sk, kind):
    """The prefill kernel at production scale: K = 8192 (128 K-tiles per split down to 16),
    grids of >= 256 tiles (every CU busy, XCD remap and GROUP_M walk over many super-rows),
    the SwiGLU epilogue, against the fp32 reference."""
    x = _bf(M, K, seed=63)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=64)
    nout = N // 2 if epi == "silu" else N
    want = ref.linear(x, w, None, epi)
    out = torch.empty(M, nout, dtype=torch.bfloat16, device=DEV)
    ws = torch.zeros(sk * M * N + 16384, dtype=torch.float32, device=DEV)
    torch.ops.bfly.gemm_with_plan(x, w, out, [kind, 0, 0, 0, 256, 256, sk], ops.EPILOGUES[epi], ws)
    _close(out, want, 2e-2, 2e-2)


TILE_CFGS = [(16, 128, 1), (16, 256, 1), (32, 128, 1), (32, 256, 1), (64, 128, 1), (64, 128, 2),
             (64, 256, 1), (64, 256, 2), (128, 128, 2), (128, 256, 2), (64, 224, 4), (64, 160, 4)]


@pytest.mark.parametrize("bm,bn,wmw", TILE_CFGS)
@pytest.mark.parametrize("epi", ["none", "silu"])
def test_gemm_tile_plans(bm, bn, wmw, epi):
    M, N, K = min(bm, 40) if bm < 128 else 200, 512 if bn in (128, 256) else 3 * bn, 1024
    x = _bf(M, K, seed=40)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=41)
    nout = N // 2 if epi == "silu" else N
    for st in (2, 3, 4):
        if st * (bm + bn) * 128 > 160 * 1024:
            continue
        for sk in (1, 3, 5):   # uneven K splits: 16 k-tiles over 3 / 5 workgroups (1..4 deep)
            out = torch.empty(M, nout, dtype=torch.bfloat16, device=DEV)
            ws = torch.zeros(sk * M * N + 16384, dtype=torch.float32, device=DEV)  # [reserved head | partials]
            torch.ops.bfly.gemm_with_plan(x, w, out, [1, st, 0, wmw, bm, bn, sk], ops.EPILOGUES[epi], ws)
            _close(out, ref.linear(x, w, epilogue=epi), 2e-2, 2e-2)


def _tuned_entries():
    import re

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "kernels", "gemm_tuned.inc")
    out = []
    for line in open(path):
        m = re.match(r"\{(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+)\}", line)
        if m:
            out.append(tuple(int(v) for v in m.groups()))
    return out


@pytest.mark.parametrize("NK", sorted({(e[0], e[1]) for e in _tuned_entries()}))
def test_every_tuned_plan_matches_fp32(NK):
    """Every entry of the measured plan table (gemm_tuned.inc: the plan the 70B / 8B / Mixtral
    projections run at each token-count bucket) through ops.linear at that bucket's M, against
    the fp32 reference; deferred (split-K slab) outputs reduced by the consumer-side reduce."""
    N, K = NK
    g = torch.Generator(device=DEV).manual_seed(N % 97)   # device-side: LM-head weights are 2 GB
    w = (torch.randn(N, K, device=DEV, generator=g) / math.sqrt(K)).to(torch.bfloat16)
    for e in _tuned_entries():
        if (e[0], e[1]) != NK:
            continue
        M = e[2]
        x = _bf(M, K, seed=M + 3)
        plan = ops.gemm_plan(M, N, K)
        # 256x256 entries (swept on big8, kind 4) run the one-wave-per-SIMD big4 (kind 6)
        assert [("skinny", "tile", "big", "dec", "big8", "mid8", "big4", "mid4").index(plan["kind"]), plan["splitk"]] == \
            [6 if e[3] == 4 else e[3], e[9]], (e, plan)
        want = x.float() @ w.float().t()
        _close(ops.linear(x, w), want, 2e-2, 2e-2)
        _close(ops.materialize(ops.linear(x, w, defer=True)), want, 2e-2, 2e-2)
        if N % 32 == 0 and N <= 65536:
            _close(ops.linear(x, w, epilogue="silu"), ref.linear(x, w, None, "silu"), 2e-2, 2e-2)


MID_CFGS = [(256, 128, 3, 3), (256, 128, 2, 6), (256, 128, 3, 4), (128, 256, 3, 3), (128, 256, 2, 4),
            (128, 128, 4, 4), (128, 128, 3, 3), (128, 128, 3, 6), (128, 128, 2, 8), (128, 128, 2, 2)]


@pytest.mark.parametrize("bm,bn,sx,st", MID_CFGS)
def test_gemm_mid8_plans(bm, bn, sx, st):
    """Mid-M 8-wave staggered GEMM (plan kind 5, activation ring sx / weight ring st): ragged M
    below and above one row tile (rows past M read as zeros through the descriptor), K-tile
    counts of 1 .. 2 x the ring depth per split (prologue / tail waits), uneven split-K, all
    epilogues, asymmetric operands."""
    N = 3 * bn
    for M, K in ((bm - 5, 1024), (bm + 9, 192), (3 * bm + 1, 4096), (7, 64 * st), (bm, 64 * (st + 1))):
        x = _bf(M, K, seed=47)
        w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=48)
        b = _bf(N, seed=49)
        for epi in ("none", "bias", "silu"):
            nout = N // 2 if epi == "silu" else N
            want = ref.linear(x, w, b if epi == "bias" else None, "silu" if epi == "silu" else "none")
            for sk in (1, 2, 3, 7):
                if K // 64 < sk:
                    continue
                out = torch.empty(M, nout, dtype=torch.bfloat16, device=DEV)
                ws = torch.zeros(sk * M * N + 16384, dtype=torch.float32, device=DEV)
                torch.ops.bfly.gemm_with_plan(x, w, out, [5, st, sx, 0, bm, bn, sk], ops.EPILOGUES[epi], ws,
                                              b if epi == "bias" else None)
                _close(out, want, 2e-2, 2e-2)


@pytest.mark.parametrize("M,N,K,plan", [(512, 1280, 8192, [5, 3, 0, 0, 128, 256, 12]),    # tp8 QKV
                                        (512, 8192, 3584, [5, 3, 0, 0, 128, 256, 2]),     # tp8 down
                                        (256, 14336, 8192, [5, 6, 2, 0, 256, 128, 2]),    # tp4 gate_up
                                        (256, 2560, 8192, [5, 6, 3, 0, 128, 128, 6])])    # tp4 QKV
def test_gemm_mid8_production(M, N, K, plan):
    """The mid-M kernel at the TP shard shapes it is tuned for (K up to 8192, >= 240
    workgroups), against the fp32 reference."""
    x = _bf(M, K, seed=57)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=58)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ws = torch.zeros(plan[6] * M * N + 16384, dtype=torch.float32, device=DEV)
    torch.ops.bfly.gemm_with_plan(x, w, out, plan, 0, ws)
    _close(out, ref.linear(x, w), 2e-2, 2e-2)


MID4_CFGS = [(128, 128, 4, 6), (128, 128, 3, 7), (128, 128, 2, 8), (256, 128, 3, 4), (256, 128, 2, 6),
             (128, 256, 4, 3), (128, 256, 2, 4)]


@pytest.mark.parametrize("bm,bn,sa,sb", MID4_CFGS)
def test_gemm_mid4_plans(bm, bn, sa, sb):
    """Mid-M one-wave-per-SIMD GEMM (plan kind 7, activation ring sa / weight ring sb): ragged M
    below and above one row tile, K-tile counts from 1 to past both rings per split (the
    per-iteration DMA wait counts of the first iterations and the clamped tail loads), uneven
    split-K, all epilogues, asymmetric operands."""
    N = 3 * bn
    for M, K in ((bm - 5, 1024), (bm + 9, 192), (3 * bm + 1, 4096), (7, 64), (bm, 64 * (sb + 2))):
        x = _bf(M, K, seed=147)
        w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=148)
        b = _bf(N, seed=149)
        for epi in ("none", "bias", "silu"):
            nout = N // 2 if epi == "silu" else N
            want = ref.linear(x, w, b if epi == "bias" else None, "silu" if epi == "silu" else "none")
            for sk in (1, 2, 3, 7):
                if K // 64 < sk:
                    continue
                out = torch.empty(M, nout, dtype=torch.bfloat16, device=DEV)
                ws = torch.zeros(sk * M * N + 16384, dtype=torch.float32, device=DEV)
                torch.ops.bfly.gemm_with_plan(x, w, out, [7, sa, sb, 0, bm, bn, sk], ops.EPILOGUES[epi], ws,
                                              b if epi == "bias" else None)
                _close(out, want, 2e-2, 2e-2)


DEC_CFGS = [(128, 224, 8, 1, 4), (128, 224, 8, 1, 3), (128, 256, 8, 1, 3), (128, 256, 4, 2, 3), (128, 128, 8, 1, 5),
            (128, 128, 4, 2, 5), (128, 160, 8, 1, 4), (128, 80, 8, 1, 6), (128, 64, 8, 1, 8), (128, 64, 4, 2, 8),
            (64, 128, 4, 2, 6), (64, 256, 4, 2, 4), (64, 224, 4, 1, 4), (64, 160, 4, 2, 5), (64, 64, 4, 2, 8)]


@pytest.mark.parametrize("bm,bn,nwm,nwn,sw", DEC_CFGS)
def test_gemm_decode_ring_plans(bm, bn, nwm, nwn, sw):
    """Decode ring GEMM (plan kind 3, separate X / W LDS rings): ragged M (< BM, and > BM so
    two row tiles share a weight panel), K-tile counts shorter than the weight ring (tail
    waits), uneven split-K, all epilogues that the tile width allows."""
    N = 3 * bn
    for M, K in ((bm - 5, 1024), (bm + 9, 192), (bm // 2, 4096)):
        x = _bf(M, K, seed=44)
        w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=45)
        b = _bf(N, seed=46)
        for epi in ("none", "bias", "silu") if (bn // nwn) % 32 == 0 else ("none", "bias"):
            nout = N // 2 if epi == "silu" else N
            want = ref.linear(x, w, b if epi == "bias" else None, "silu" if epi == "silu" else "none")
            for sk in (1, 3):
                if K // 64 < 2 * sk:
                    continue
                out = torch.empty(M, nout, dtype=torch.bfloat16, device=DEV)
                ws = torch.zeros(sk * M * N + 16384, dtype=torch.float32, device=DEV)
                torch.ops.bfly.gemm_with_plan(x, w, out, [3, sw, nwm * nwn, nwm, bm, bn, sk], ops.EPILOGUES[epi], ws,
                                              b if epi == "bias" else None)
                _close(out, want, 2e-2, 2e-2)


@pytest.mark.parametrize("mt,nt,wk", [(1, 1, 4), (1, 2, 1), (1, 4, 4), (2, 2, 2), (2, 4, 1), (4, 1, 4), (4, 2, 1), (4, 4, 4), (3, 2, 2)])
def test_gemm_skinny_plans(mt, nt, wk):
    M, N, K = 16 * mt - 3, 512, 1024
    x = _bf(M, K, seed=42)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=43)
    for epi in ("none", "silu") if nt % 2 == 0 else ("none",):
        nout = N // 2 if epi == "silu" else N
        for sk in (1, 2):
            out = torch.empty(M, nout, dtype=torch.bfloat16, device=DEV)
            ws = torch.zeros(sk * M * N + 16384, dtype=torch.float32, device=DEV)  # [reserved head | partials]
            torch.ops.bfly.gemm_with_plan(x, w, out, [0, mt, nt, wk, 0, 0, sk], ops.EPILOGUES[epi], ws)
            _close(out, ref.linear(x, w, epilogue=epi), 2e-2, 2e-2)


@pytest.mark.parametrize("M,N,K", [(64, 8192, 8192), (7, 1280, 8192), (64, 10240, 8192)])
def test_gemm_deferred_reduce_fusions(M, N, K):
    """A split-K GEMM left unreduced (Partial) must give the same result through every fused
    consumer as the plain GEMM followed by the unfused op."""
    x = _bf(M, K, seed=70)
    w = _bf(N, K, scale=1.0 / math.sqrt(K), seed=71)
    full = ops.linear(x, w)
    p = ops.linear(x, w, defer=True)
    if not isinstance(p, ops.Partial):
        pytest.skip("plan does not split K for this shape")
    got = ops.linear(x, w, defer=True).materialize()
    torch.testing.assert_close(got, full, atol=0, rtol=0)
    # (fused consumers may sum the slabs in another association order under -ffast-math:
    # equal up to one bf16 rounding step)
    # add + rmsnorm with the reduce fused in
    if N == 8192:
        wn = _bf(N, seed=72)
        r0 = _bf(M, N, seed=73)
        ra, rb = r0.clone(), r0.clone()
        ya = ops.rms_norm(full, wn, 1e-5, residual=ra)
        yb = ops.rms_norm(ops.linear(x, w, defer=True), wn, 1e-5, residual=rb)
        torch.testing.assert_close(rb, ra, atol=1e-2, rtol=1e-2)
        torch.testing.assert_close(yb, ya, atol=2e-2, rtol=2e-2)
    # rope + KV append with the reduce fused in
    if N == 10240:
        hq, hkv, D, BS = 64, 8, 128, 32
        cos, sin = ref.rope_tables(D, 4096, 500000.0)
        cos, sin = cos.to(DEV), sin.to(DEV)
        pos = torch.randint(0, 4000, (M,), dtype=torch.int32, device=DEV)
        slots = torch.randperm(8 * BS, device=DEV)[:M].to(torch.int32)
        kc = [torch.zeros(8, hkv, BS, D, dtype=torch.bfloat16, device=DEV) for _ in range(2)]
        vc = [torch.zeros(8, hkv, D, BS, dtype=torch.bfloat16, device=DEV) for _ in range(2)]
        qa = ops.rope_kv(full.clone(), pos, cos, sin, hq, hkv, slots, kc[0], vc[0])
        qb = ops.rope_kv(ops.linear(x, w, defer=True), pos, cos, sin, hq, hkv, slots, kc[1], vc[1])
        torch.testing.assert_close(qb, qa, atol=2e-2, rtol=2e-2)
        torch.testing.assert_close(kc[1], kc[0], atol=2e-2, rtol=2e-2)
        torch.testing.assert_close(vc[1], vc[0], atol=2e-2, rtol=2e-2)


# (M, hidden, consumer N, epilogue, deferred): Llama-3-70B QKV (tile plan, split-K slabs) and
# gate/up (tile, SiLU), Llama-3-8B QKV (decode-ring plan), a biased consumer, ragged row counts
ROWSCALE_CASES = [(64, 8192, 10240, "none", True), (64, 8192, 57344, "silu", False),
                  (64, 4096, 6144, "none", True), (61, 4096, 28672, "silu", False),
                  (200, 8192, 1024, "bias", False), (33, 8192, 10240, "none", False),
                  # production decode batches 65-256: consumers on the mid-M plans
                  # (kinds 5 / 7), whose epilogue applies the row scale
                  (128, 8192, 10240, "none", True), (256, 4096, 6144, "none", True),
                  (256, 4096, 28672, "silu", False), (128, 8192, 57344, "silu", False),
                  (250, 8192, 10240, "none", False)]
MID_ROWSCALE = {(128, 8192, 10240), (256, 4096, 6144), (256, 4096, 28672), (128, 8192, 57344),
                (250, 8192, 10240)}


@pytest.mark.parametrize("M,H,N,epi,defer", ROWSCALE_CASES)
@pytest.mark.parametrize("src", ["slabs", "bf16"])
def test_rms_norm_rows_with_rowscale_consumer(M, H, N, epi, defer, src):
    """Row-split add + RMSNorm (y = x * g, partial sums of squares) followed by a GEMM that
    applies the 1/rms row scale in its epilogue == fp32 add + RMSNorm + GEMM; the residual
    update is bit-identical to the one-workgroup-per-row kernel's."""
    if (M, H, N) in MID_ROWSCALE:
        # these must run the mid-M kernels with the row-scale epilogue, not skip
        assert ops.gemm_plan(M, N, H)["kind"] in ("mid8", "mid4"), ops.gemm_plan(M, N, H)
        assert ops.rowscale_ok(M, N, H, epi)
    if not ops.rowscale_ok(M, N, H, epi):
        pytest.skip(f"plan for {M}x{N}x{H} takes no row scale")
    K0 = 8192   # long enough that the producer GEMM splits K (slab input)
    x0 = _bf(M, K0, seed=80)
    w0 = _bf(H, K0, scale=1.0 / math.sqrt(K0), seed=81)
    g = (1.0 + 0.5 * _bf(H, seed=82).float()).to(torch.bfloat16)
    W = _bf(N, H, scale=1.0 / math.sqrt(H), seed=83)
    b = _bf(N, seed=84) if epi == "bias" else None
    r0 = _bf(M, H, seed=85)
    delta = ops.linear(x0, w0)

    def make_src():
        if src == "bf16":
            return delta
        p = ops.linear(x0, w0, defer=True)
        if not isinstance(p, ops.Partial):
            pytest.skip("producer plan does not split K")
        return p

    ra, rb = r0.clone(), r0.clone()
    ya = ops.rms_norm(make_src(), g, 1e-5, residual=ra)
    rn = ops.rms_norm(make_src(), g, 1e-5, residual=rb, rows=True)
    assert isinstance(rn, ops.RowNormed)
    torch.testing.assert_close(rb, ra, atol=0, rtol=0)
    got = ops.linear(rn, W, bias=b, epilogue="silu" if epi == "silu" else "none", defer=defer)
    got = ops.materialize(got)
    # fp32 reference from the stored bf16 residual
    s = rb.float()
    yn = s * torch.rsqrt(s.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    want = ref.linear(yn.cpu(), W.float().cpu(), None if b is None else b.float().cpu(),
                      "silu" if epi == "silu" else "none")
    _close(got, want, 3e-2, 3e-2)
    # and against the existing (normalise, then GEMM) path
    base = ops.linear(ya, W, bias=b, epilogue="silu" if epi == "silu" else "none")
    _close(got, base, 3e-2, 3e-2)


@pytest.mark.parametrize("T,E,El,e0,k,H,F", [(300, 8, 8, 0, 2, 512, 256), (64, 8, 4, 4, 2, 256, 128),
                                           (1000, 8, 2, 2, 2, 256, 128), (5, 8, 8, 0, 2, 256, 128)])
def test_moe_sparse_ffn(T, E, El, e0, k, H, F):
    """Routed (permute + grouped GEMM + combine) expert FFN against the fp32 reference, with a
    local expert subset (EP shard) and tokens routed elsewhere."""
    x = _bf(T, H, seed=80)
    wr = _bf(E, H, seed=81)
    _, ids, w = ops.moe_route(x, wr, k)
    gu = _bf(El * 2 * F, H, scale=1.0 / math.sqrt(H), seed=82)
    dn = _bf(H, El * F, scale=1.0 / math.sqrt(F), seed=83)
    got = ops.moe_sparse_ffn(x, ids, w, gu, dn, e0, El, F)
    want = ref.moe_sparse_ffn(x.cpu().float(), ids.cpu(), w.cpu(), gu.cpu().float(), dn.cpu().float(), e0, El, F)
    _close(got, want, 3e-2, 3e-2)
    # the dense path (all local experts on every token, gate-scaled) computes the same function
    gates = torch.zeros(T, E, device=DEV).scatter_(1, ids.long(), w)
    h = ops.linear(x, gu, epilogue="silu")
    ops.moe_gate_scale_(h, gates, e0, El)
    dense = ops.linear(h, dn)
    _close(got, dense, 3e-2, 3e-2)


@pytest.mark.parametrize("T,El,e0,H,F,skew", [(4096, 8, 0, 512, 256, False), (3000, 8, 0, 256, 512, True),
                                                (4096, 2, 2, 512, 256, True), (2600, 4, 4, 1024, 256, False)])
def test_moe_sparse_ffn_big_tile(T, El, e0, H, F, skew):
    """Prefill-scale routing (>= 256 rows per local expert): the expert GEMMs run the 8-phase
    256x256 tile over the device tile list (gathered token rows, expert weight slices, ragged
    last tiles), with skewed loads and an expert that gets no rows, against the fp32 reference
    and the dense gate-scaled path."""
    E, k = 8, 2
    g = torch.Generator().manual_seed(90 + T)
    if skew:   # experts 0-2 take most pairs, expert 5 none
        p = torch.tensor([0.3, 0.25, 0.2, 0.08, 0.08, 0.0, 0.05, 0.04])
    else:
        p = torch.full((E,), 1.0 / E)
    ids = torch.stack([torch.multinomial(p, k, replacement=False, generator=g) for _ in range(T)]).to(torch.int32)
    w = torch.rand(T, k, generator=g)
    w = (w / w.sum(1, keepdim=True)).float()
    x = _bf(T, H, seed=84)
    gu = _bf(El * 2 * F, H, scale=1.0 / math.sqrt(H), seed=85)
    dn = _bf(H, El * F, scale=1.0 / math.sqrt(F), seed=86)
    ids_d, w_d = ids.to(DEV), w.to(DEV)
    got = ops.moe_sparse_ffn(x, ids_d, w_d, gu, dn, e0, El, F)
    want = ref.moe_sparse_ffn(x.cpu().float(), ids, w, gu.cpu().float(), dn.cpu().float(), e0, El, F)
    _close(got, want, 3e-2, 3e-2)
    os.environ["BFLY_MOE_BIG_TILE"] = "0"
    try:
        ops._BIG_MOE = False
        base = ops.moe_sparse_ffn(x, ids_d, w_d, gu, dn, e0, El, F)
    finally:
        ops._BIG_MOE = True
        os.environ.pop("BFLY_MOE_BIG_TILE")
    _close(got, base, 2e-2, 2e-2)


@pytest.mark.parametrize("cap,counts,El", [(96, [0, 37, 96, 5], 1), (256, [200, 3, 0, 17, 250, 1, 90, 64], 2)])
def test_moe_sparse_ffn_block_counts(cap, counts, El):
    """EP prefill receive buffer: blocks of `cap` rows of which only the first counts[b] are
    valid (device-resident counts, rows beyond hold stale garbage with live expert ids). The
    valid rows must equal the fp32 reference over exactly those rows; nothing else is computed
    or written (the invalid output rows keep their poison)."""
    H, F, E, k = 512, 1024, 8, 2
    nb = len(counts)
    T = nb * cap
    x = _bf(T, H, seed=95)
    _, ids, w = ops.moe_route(x, _bf(E, H, seed=96), k)
    gu = _bf(El * 2 * F, H, scale=1.0 / math.sqrt(H), seed=97)
    dn = _bf(H, El * F, scale=1.0 / math.sqrt(F), seed=98)
    cnt = torch.tensor(counts, dtype=torch.int32, device=DEV)
    got = ops.moe_sparse_ffn(x, ids, w, gu, dn, 1, El, F, block_counts=(cnt, cap))
    valid = torch.cat([torch.arange(cap) < c for c in counts])
    want = ref.moe_sparse_ffn(x.cpu().float()[valid], ids.cpu()[valid], w.cpu()[valid], gu.cpu().float(),
                              dn.cpu().float(), 1, El, F)
    _close(got[valid.to(DEV)], want, 3e-2, 3e-2)


@pytest.mark.parametrize("T,El,e0,H,F,pad,expect", [(64, 1, 3, 1024, 4096, 0, None),     # bm 128, split-K
                                                    (200, 2, 2, 512, 2048, 0, None),     # bm 128, 2 experts
                                                    (512, 1, 5, 1024, 4096, 384, 256),   # EP dispatch padding
                                                    (96, 4, 0, 512, 4096, 0, None)])     # bm 64, split-K
def test_moe_sparse_ffn_decode_shapes(T, El, e0, H, F, pad, expect):
    """Decode-sized routed expert batches: 128-row expert tiles (weights read once, non-temporal),
    the split-K grouped down projection whose f32 slabs are reduced inside the weighted combine
    (moe_combine_slabs), and EP-dispatch padding rows (expert ids -1) that must cost and change
    nothing — all against the fp32 reference."""
    E, k = 8, 2
    x = _bf(T, H, seed=90)
    wr = _bf(E, H, seed=91)
    _, ids, w = ops.moe_route(x, wr, k)
    if pad:
        ids[T - pad:] = -1            # padding slots of the fixed-capacity dispatch
    gu = _bf(El * 2 * F, H, scale=1.0 / math.sqrt(H), seed=92)
    dn = _bf(H, El * F, scale=1.0 / math.sqrt(F), seed=93)
    exp = expect if expect is not None else T * k
    bm = 128 if exp >= 96 * El else 64
    assert ops.moe_down_splits(exp, El, H, F, bm) > 1
    got = ops.moe_sparse_ffn(x, ids, w, gu, dn, e0, El, F, expected_slots=expect)
    want = ref.moe_sparse_ffn(x.cpu().float(), ids.cpu(), w.cpu(), gu.cpu().float(), dn.cpu().float(), e0, El, F)
    _close(got, want, 3e-2, 3e-2)
    if pad:
        assert got[T - pad:].abs().max().item() == 0.0


@pytest.mark.parametrize("causal", [True, False])
def test_attn_prefill_lse_and_key_offsets(causal):
    """K3 with LSE output, and (non-causal) keys taken from other rows than the queries — the
    ring-attention step of context parallelism."""
    D, Hq, Hkv = 128, 8, 2
    lq, lk = [1, 70, 300], ([1, 70, 300] if causal else [5, 0, 129])
    cu = torch.tensor([0] + list(torch.tensor(lq).cumsum(0)), dtype=torch.int32, device=DEV)
    cuk = torch.tensor([0] + list(torch.tensor(lk).cumsum(0)), dtype=torch.int32, device=DEV)
    q = _bf(sum(lq), Hq, D, seed=80)
    k, v = _bf(sum(lk), Hkv, D, seed=81), _bf(sum(lk), Hkv, D, seed=82)
    kw = {} if causal else {"cu_seqlens_k": cuk}
    o, lse = ops.attn_prefill(q, k, v, cu, max(lq), 0.088, causal, return_lse=True, **kw)
    ro, rl = ref.attn_prefill(q.cpu(), k.cpu(), v.cpu(), cu.cpu(), max(lq), 0.088, causal, return_lse=True,
                              **({} if causal else {"cu_seqlens_k": cuk.cpu()}))
    _close(o, ro, 2e-2, 2e-2)
    fin = torch.isfinite(rl)
    assert torch.equal(torch.isfinite(lse.cpu()), fin)
    _close(lse.cpu()[fin], rl[fin], 2e-3, 1e-3)


def test_attn_lse_merge():
    T, H, D = 37, 8, 128
    acc = torch.randn(T, H, D, device=DEV)
    al = torch.randn(T, H, device=DEV) * 3
    al[3, :] = float("-inf")
    o = _bf(T, H, D, seed=83)
    lse = torch.randn(T, H, device=DEV) * 3
    lse[5, 2] = float("-inf")
    lse[3, 1] = float("-inf")
    a2, l2 = acc.cpu().clone(), al.cpu().clone()
    ops.attn_lse_merge_(acc, al, o, lse)
    ref.attn_lse_merge_(a2, l2, o.cpu(), lse.cpu())
    _close(acc, a2, 1e-3, 1e-3)
    fin = torch.isfinite(l2)
    assert torch.equal(torch.isfinite(al.cpu()), fin)
    _close(al.cpu()[fin], l2[fin], 1e-4, 1e-4)


# ---- FP8 (e4m3) KV cache ----------------------------------------------------------------
F8 = torch.float8_e4m3fn


@pytest.mark.parametrize("Hq,Hkv", [(8, 1), (32, 8)])
def test_attn_decode_fp8_cache(Hq, Hkv):
    """Decode attention over an FP8 cache == the fp32 reference over the same FP8 values."""
    D, BS = 128, 32
    lens = [1, 33, 300, 900]
    B = len(lens)
    mb = (max(lens) + BS - 1) // BS
    nblk = B * mb + 2
    kc = (_bf(nblk, Hkv, BS, D, seed=60) * 3).to(F8)
    vc = (_bf(nblk, Hkv, D, BS, seed=61) * 3).to(F8)
    bt = torch.randperm(nblk)[: B * mb].view(B, mb).to(torch.int32).to(DEV)
    ctx = torch.tensor(lens, dtype=torch.int32, device=DEV)
    q = _bf(B, Hq, D, seed=62)
    scale = 1.0 / math.sqrt(D)
    want = ref.attn_decode(q, kc, vc, bt, ctx, scale)
    o = ops.attn_decode(q, kc, vc, bt, ctx, scale, max(lens))
    _close(o, want, 2e-2, 2e-2)
    # and close to attention over the unquantized values (e4m3: ~3 significant bits)
    o16 = ops.attn_decode(q, kc.to(torch.bfloat16), vc.to(torch.bfloat16), bt, ctx, scale, max(lens))
    _close(o, o16, 2e-2, 2e-2)


def test_rope_kv_and_kv_append_fp8_cache():
    """The kernels store torch's bf16 -> float8_e4m3fn conversion (RNE, clamped to +-448) of
    the rotated K and of V, at the paged (K row / transposed V) positions."""
    D, BS, Hq, Hkv, T = 128, 32, 8, 2, 37
    qkv = _bf(T, (Hq + 2 * Hkv) * D, seed=63) * 40          # some values past the e4m3 range
    pos = torch.randint(0, 500, (T,), dtype=torch.int32).to(DEV)
    inv = 1.0 / (500000 ** (torch.arange(0, D, 2).float() / D))
    ang = torch.arange(1024).float()[:, None] * inv[None]
    cos, sin = ang.cos().to(DEV), ang.sin().to(DEV)
    nblk = 4
    slots = torch.randperm(nblk * BS)[:T].to(torch.int32).to(DEV)
    kc = torch.zeros(nblk, Hkv, BS, D, dtype=F8, device=DEV)
    vc = torch.zeros(nblk, Hkv, D, BS, dtype=F8, device=DEV)
    out = ops.rope_kv(qkv.clone(), pos, cos, sin, Hq, Hkv, slots, kc, vc)
    k = out[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D).float().clamp(-448, 448).to(F8)
    v = out[:, (Hq + Hkv) * D:].view(T, Hkv, D).float().clamp(-448, 448).to(F8)
    sl = slots.long()
    blk, off = sl // BS, sl % BS
    assert torch.equal(kc[blk, :, off, :].view(torch.uint8), k.view(torch.uint8))
    assert torch.equal(vc[blk, :, :, off].view(torch.uint8), v.view(torch.uint8))
    kc2, vc2 = torch.zeros_like(kc), torch.zeros_like(vc)
    kk = out[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D)
    vv = out[:, (Hq + Hkv) * D:].view(T, Hkv, D)
    ops.kv_append(kk, vv, slots, kc2, vc2)
    assert torch.equal(kc2.view(torch.uint8), kc.view(torch.uint8))
    assert torch.equal(vc2.view(torch.uint8), vc.view(torch.uint8))


@pytest.mark.parametrize("T,cap,ep,El,with_slots", [(64, 64, 8, 1, False), (37, 48, 4, 2, True), (5, 8, 2, 4, True)])
def test_ep_pack_and_combine(T, cap, ep, El, with_slots):
    """Fixed-capacity EP dispatch packing (ep_pack_kernel) equals the reference layout exactly
    (row positions, copied rows, int32-bit expert ids, weights, empty metadata rows), and the
    return combine sums each token's returned rows."""
    E, k, H = ep * El, 2, 256
    x = _bf(T, H, seed=95)
    wr = _bf(E, H, seed=96)
    _, ids, w = ops.moe_route(x, wr, k)
    slots = None
    if with_slots:
        slots = torch.arange(T, dtype=torch.int32, device=DEV)
        slots[::3] = -1                     # graph padding rows: route nowhere
    send, meta, slot = ops.ep_pack(x, ids, w, slots, El, ep, cap)
    rs, rm, rslot = ref.ep_pack(x.cpu(), ids.cpu(), w.cpu(), None if slots is None else slots.cpu(), El, ep, cap)
    assert torch.equal(slot.cpu(), rslot)
    sent = rslot[rslot >= 0].long()
    assert torch.equal(send.cpu()[sent], rs[sent])
    assert torch.equal(meta.cpu().view(torch.int32)[:, :k], rm.view(torch.int32)[:, :k])
    assert torch.equal(meta.cpu()[:, k:], rm[:, k:])
    back = _bf(ep * cap, H, seed=97)
    got = ops.ep_combine(back, slot)
    want = ref.ep_combine(back.cpu(), rslot)
    _close(got, want, 1e-2, 1e-2)


def _attn_ref_gpu(q, k, v, cu, scale, heads):
    """fp32 causal attention on the GPU for the listed query heads (row chunks of 2048)."""
    G = q.shape[1] // k.shape[1]
    out = {}
    for h in heads:
        kh = h // G
        parts = []
        for i in range(len(cu) - 1):
            a, b = int(cu[i]), int(cu[i + 1])
            qh, kk, vv = q[a:b, h].float(), k[a:b, kh].float(), v[a:b, kh].float()
            for r0 in range(0, b - a, 2048):
                r1 = min(b - a, r0 + 2048)
                s = (qh[r0:r1] @ kk[:r1].t()) * scale
                rows = torch.arange(r0, r1, device=q.device)[:, None]
                s = s.masked_fill(torch.arange(r1, device=q.device)[None, :] > rows, float("-inf"))
                parts.append(torch.softmax(s, -1) @ vv[:r1])
        out[h] = torch.cat(parts)
    return out


@pytest.mark.parametrize("lens,Hq,Hkv,heads", [
    ([1024] * 4, 64, 8, [0, 7, 8, 63]),          # bench shape: 1024-token prompts, 64 q / 8 kv heads
    ([4096], 64, 8, [0, 9, 35, 63]),
    ([16384], 16, 2, [0, 15]),                    # long context: the ring in steady state
    ([3000, 1, 777, 4100, 64, 2], 16, 2, [1, 8, 14]),   # varlen mix, ragged block ends
])
def test_attn_prefill_long_vs_fp32(lens, Hq, Hkv, heads):
    """K3 at the prompt lengths the engine and bench run (1k-16k): every query block of the
    heaviest-first causal order, the multi-stage LDS ring in steady state and ragged ends,
    against an fp32 reference of the same bf16 inputs."""
    D = 128
    T = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    g = torch.Generator(device=DEV).manual_seed(7)
    q = (torch.randn(T, Hq, D, device=DEV, generator=g) * 1.5).to(torch.bfloat16)
    k = (torch.randn(T, Hkv, D, device=DEV, generator=g) * 1.5).to(torch.bfloat16)
    v = torch.randn(T, Hkv, D, device=DEV, generator=g).to(torch.bfloat16)
    scale = 1.0 / math.sqrt(D)
    o = ops.attn_prefill(q, k, v, cu, max(lens), scale, True)
    want = _attn_ref_gpu(q, k, v, cu, scale, heads)
    for h in heads:
        got = o[:, h].float()
        err = (got - want[h]).abs().max().item()
        rel = ((got - want[h]).norm() / want[h].norm()).item()
        assert err < 3e-2 and rel < 1e-2, (h, err, rel)


@pytest.mark.parametrize("epi", ["none", "silu", "bias"])
def test_linear_large_m_prefill_path(epi):
    """Prefill-sized GEMMs (M > 256, an M tail) run the 256x256 one-wave-per-SIMD kernel for
    every epilogue; there is no library fallback left in linear()."""
    assert ops.gemm_plan(4100, 1024, 512)["kind"] == "big4"
    x, w = _bf(4100, 512, seed=90), _bf(1024, 512, seed=91, scale=0.05)
    b = _bf(1024, seed=92) if epi == "bias" else None
    own = ops.linear(x, w, bias=b, epilogue="none" if epi == "bias" else epi)
    want = ref.linear(x.float(), w.float(), b.float() if b is not None else None,
                      epilogue="none" if epi == "bias" else epi)
    _close(own, want, 3e-2, 3e-2)


def test_sample_check_finite():
    """The NaN guard inside the sampling kernels: rows with an Inf / NaN logit give id -1 and
    score +inf, every other row samples exactly as without the check."""
    lg = _bf(6, 50000, seed=95)
    lg[1, 777] = float("nan")
    lg[4, 49999] = float("inf")
    temps = torch.tensor([0.0, 0.0, 0.7, 0.0, 1.0, 0.9], device=DEV)
    seeds = torch.arange(6, dtype=torch.int64, device=DEV) * 7 + 1
    ids, sc = ops.sample(lg, temps, seeds, check_finite=True)
    ids0, sc0 = ops.sample(lg, temps, seeds)
    ids, sc, ids0 = ids.cpu(), sc.cpu(), ids0.cpu()
    assert ids[1] == -1 and ids[4] == -1 and torch.isinf(sc[1]) and torch.isinf(sc[4])
    keep = [0, 2, 3, 5]
    assert torch.equal(ids[keep], ids0[keep])
    rid, _ = ref.sample(lg.cpu(), temps.cpu(), seeds.cpu(), 0, None, True)
    assert torch.equal(rid.cpu(), ids)




def test_gather_rows_matches_index_select():
    """ops.gather_rows (elementwise.hip): bf16 hidden rows by int64 indices (final-token rows),
    int32 single-column rows with -1 holes keeping their pre-filled values (pipeline input ids),
    and odd-width f32 rows from a strided view (4-byte fallback path)."""
    g = torch.Generator(device=DEV).manual_seed(5)
    src = torch.randn(50, 8192, device=DEV, generator=g).to(torch.bfloat16)
    idx = torch.tensor([49, 0, 7, 7, 31], dtype=torch.int64, device=DEV)
    assert torch.equal(ops.gather_rows(src, idx), src.index_select(0, idx))
    ids = torch.arange(100, 140, dtype=torch.int32, device=DEV).view(-1, 1)
    sel = torch.tensor([3, -1, 0, 39, -1, 5], dtype=torch.int32, device=DEV)
    out = torch.full((6, 1), -7, dtype=torch.int32, device=DEV)
    ops.gather_rows(ids, sel, out=out)
    assert out.flatten().tolist() == [103, -7, 100, 139, -7, 105]
    big = torch.randn(20, 8, device=DEV, generator=g)
    view = big[:, 1:4]                                   # 3 words per row, row stride 8
    want = view.index_select(0, idx.clamp(max=19))
    assert torch.equal(ops.gather_rows(view, idx.clamp(max=19)), want)


@pytest.mark.parametrize("tp", [2, 4, 8])
def test_sample_pack_merge_matches_torch(tp):
    """TP sampling merge kernels (sample.hip) against the torch stack / argmax / gather they
    replace: best score per row, lowest rank on ties, ids exact through f32."""
    rows = 37
    g = torch.Generator(device=DEV).manual_seed(tp)
    scores = [torch.randn(rows, device=DEV, generator=g) for _ in range(tp)]
    scores[1][:5] = scores[0][:5]                        # ties go to the lower rank
    scores[tp - 1][7] = float("inf")                     # a non-finite row's +inf wins
    ids = [torch.randint(0, 128256, (rows,), dtype=torch.int32, device=DEV, generator=g) for _ in range(tp)]
    allp = torch.stack([ops.sample_pack(s, i) for s, i in zip(scores, ids)])
    assert torch.equal(allp, torch.stack([ref.sample_pack(s, i) for s, i in zip(scores, ids)]))
    assert torch.equal(ops.sample_merge(allp), ref.sample_merge(allp))


def test_runtime_fills():
    """ops.zero_ / fill32_ (runtime memsets that replace torch fill kernels on serving paths)."""
    t = torch.randn(1000, device=DEV)
    ops.zero_(t)
    assert int((t != 0).sum()) == 0
    u = torch.zeros(77, dtype=torch.int32, device=DEV)
    torch.ops.bfly.fill32_(u[10:20], -2 ** 31)
    assert u[10:20].tolist() == [-2 ** 31] * 10 and int(u[:10].abs().sum() + u[20:].abs().sum()) == 0


@pytest.mark.parametrize("causal", [True, False])
def test_attn_prefill_is_deterministic(causal):
    """Launch-to-launch bit equality of the persistent flash prefill on ragged multi-tile
    sequences. Regression test for an MFMA -> inline-asm read hazard (the row max read the
    S accumulators before their write-back on some waves of some launches: finite outputs
    that differed by rounding from launch to launch on every unmasked tile)."""
    torch.manual_seed(0)
    lens = [72, 39, 1, 300, 1030]
    T, Hq, Hkv = sum(lens), 16, 4
    q = torch.randn(T, Hq, 128, device="cuda").to(torch.bfloat16)
    kv = torch.randn(T, 2 * Hkv, 128, device="cuda").to(torch.bfloat16)
    cu = torch.tensor([0] + torch.tensor(lens).cumsum(0).tolist(), dtype=torch.int32, device="cuda")
    outs = [ops.attn_prefill(q, kv[:, :Hkv], kv[:, Hkv:], cu, max(lens), 128 ** -0.5, causal).clone()
            for _ in range(12)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def _same_every_launch(fn, n=8):
    outs = []
    for _ in range(n):
        r = fn()
        outs.append(tuple(t.clone() for t in (r if isinstance(r, tuple) else (r,))))
    torch.cuda.synchronize()
    return all(all(torch.equal(a, b) for a, b in zip(o, outs[0])) for o in outs[1:])


@pytest.mark.parametrize("kv_dtype", ["bf16", "fp8"])
def test_hot_kernels_are_deterministic(kv_dtype):
    """Launch-to-launch bit equality of the other hot kernels (the class of bug the flash
    prefill hazard was): paged-prefix prefill (register kernel for one sequence, LDS kernel for
    several), decode attention with and without context splits, split-K decode / prefill GEMMs
    with the SiLU epilogue, the row-split add+RMSNorm."""
    scale = 1.0 / math.sqrt(128)
    q, kc, vc, tables, cu, pos, mq = _paged_chunk_case(8, 2, kv_dtype)
    assert _same_every_launch(lambda: ops.attn_prefill_paged(q, kc, vc, tables, cu, pos, mq, scale))
    q1, kc1, vc1, t1, cu1, pos1, mq1 = _paged_chunk_case(64, 8, kv_dtype, seed=60, pre=(700,), chunk=(129,))
    assert _same_every_launch(lambda: ops.attn_prefill_paged(q1, kc1, vc1, t1, cu1, pos1, mq1, scale))
    # decode over the same pages: one split and several
    B = tables.shape[0]
    ctx = torch.tensor([p + c for p, c in zip((0, 40, 95, 700, 31), (37, 1, 50, 16, 129))], dtype=torch.int32,
                       device=DEV)
    qd = _bf(B, 8, 128, seed=71)
    for part in (0, 64):
        assert _same_every_launch(lambda: ops.attn_decode(qd, kc, vc, tables, ctx, scale, int(ctx.max()), part))
    if kv_dtype == "fp8":
        return
    for M, N, K, epi in ((64, 2048, 4096, "silu"), (64, 1024, 8192, "none"), (300, 512, 4096, "none"),
                         (1024, 1024, 2048, "silu")):
        x, w = _bf(M, K, seed=M + K), _bf(N, K, seed=N) * 0.05
        assert _same_every_launch(lambda: ops.linear(x, w, epilogue=epi)), (M, N, K, epi)
    h, g, res = _bf(64, 8192, seed=3), _bf(8192, seed=4), _bf(64, 8192, seed=5)
    assert _same_every_launch(lambda: ops.rms_norm(h, g, 1e-5, residual=res.clone(), rows=True).y)
