"""butterfly_amd ops: hand-written HIP/CDNA4 kernels bound as torch.ops.bfly.*.

GPU tensors always run the HIP kernels from the in-tree `butterfly_amd/_C.so`; if that
library is missing or fails to load, every GPU call raises (no silent eager fallback).
CPU tensors run `ops.reference` (the CPU/gloo plumbing path and the numerics oracle).

Workspaces (split-K GEMM partials, split-KV decode partials, sampling partials) come from a
per-device arena that the engine sizes before hipGraph capture (`reserve_workspace`), so
captured steps never allocate.
"""
from __future__ import annotations

import os
import threading
from typing import Optional
from pathlib import Path

import torch

from . import reference as ref
from .reference import SILU_INTERLEAVE, interleave_gate_up, rope_tables, split_gate_up  # noqa: F401

_LIB_PATH = Path(__file__).resolve().parent.parent / "_C.so"
_loaded = False
_load_error: str | None = None

EPILOGUES = {"none": 0, "bias": 1, "silu": 2}
DECODE_PART_TOKENS = 0   # 0 = pick the context split per call (attn_decode_part_tokens)


def load_library(path: str | os.PathLike | None = None) -> bool:
    """Load the HIP kernel library (idempotent). Returns True on success."""
    global _loaded, _load_error
    if _loaded:
        return True
    # BFLY_KERNEL_LIB: another build of the kernel library (same-box A/B runs of kernel changes)
    p = Path(path) if path else Path(os.environ.get("BFLY_KERNEL_LIB") or _LIB_PATH)
    if not p.exists():
        _load_error = f"{p} not built (run `python -m butterfly_amd._build`)"
        return False
    try:
        torch.ops.load_library(str(p))
        _loaded = True
        _load_error = None
    except Exception as e:  # pragma: no cover - depends on the environment
        _load_error = f"failed to load {p}: {e}"
    return _loaded


def require_library() -> None:
    """Raise unless the HIP kernel library is loaded (GPU-only features call this)."""
    if not load_library():
        raise RuntimeError(f"butterfly_amd HIP kernels unavailable: {_load_error}")


def native_available() -> bool:
    return load_library()


def library_path() -> str:
    return str(_LIB_PATH)


_FORCE_REF = False


class reference_mode:
    """Route every op to its fp32 PyTorch reference (ops/reference.py) even for GPU tensors:
    tests build an fp32 reference model on the same GPU as the kernel model (full-size layers
    whose CPU reference would take minutes). Not thread-scoped; tests only."""

    def __enter__(self):
        global _FORCE_REF
        self._prev, _FORCE_REF = _FORCE_REF, True
        return self

    def __exit__(self, *exc):
        global _FORCE_REF
        _FORCE_REF = self._prev
        return False


def _gpu(t: torch.Tensor) -> bool:
    if not t.is_cuda or _FORCE_REF:
        return False
    if not load_library():
        raise RuntimeError(f"butterfly_amd HIP kernels unavailable: {_load_error}")
    return True


# ---------------------------------------------------------------------------------------
# Workspace arena
# ---------------------------------------------------------------------------------------
class _Arena:
    """Named scratch buffers reused by every kernel call (split-K slabs, decode-attention
    partials, MoE slot maps and tile lists, sampling pairs). Buffers are shared by the threads
    of a process (an engine built on one thread and stepped on another reuses them) unless a
    thread sets its own scope (`arena_scope`): several ranks driven from threads of ONE process
    (the loopback backend, parallel/fake.py) must never share e.g. a MoE tile list, or one
    rank's moe_align would steer the other's grouped GEMM outside its own activations."""

    def __init__(self):
        self.bufs: dict[tuple, torch.Tensor] = {}
        self.frozen = False
        # buffers replaced by a larger one stay allocated: a hipGraph captured earlier still
        # reads / writes the old address (freeing it would hand that memory to someone else)
        self.retired: list = []

    def get(self, device, name: str, numel: int, dtype, zero: bool = False) -> torch.Tensor:
        key = (str(device), name, dtype, getattr(_scope, "name", None))
        buf = self.bufs.get(key)
        if buf is None or buf.numel() < numel:
            if self.frozen or (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
                raise RuntimeError(
                    f"workspace '{name}' needs {numel} elements but is frozen/capturing; "
                    "call ops.reserve_workspace() before capture")
            if buf is not None:
                self.retired.append(buf)
            buf = torch.empty(max(numel, 1), dtype=dtype, device=device)
            if zero:
                zero_(buf)
            self.bufs[key] = buf
        return buf


def zero_(t: torch.Tensor) -> torch.Tensor:
    """t.zero_() through the runtime's memset on the GPU (keeps torch kernels out of traces)."""
    if t.is_cuda and load_library():
        torch.ops.bfly.zero_(t)
    else:
        t.zero_()
    return t


# Output poisoning (`set_poison`): every op output is allocated filled with NaN
# (floating point) or a negative sentinel (integers) instead of left uninitialised, so an
# element a kernel forgot to write shows up in the comparison against the unpoisoned run.
_POISON = os.environ.get("BFLY_POISON_OUTPUTS", "0").strip().lower() in ("1", "true", "yes", "on")
# MoE prefill expert GEMMs on the 256x256 8-phase tile (BFLY_MOE_BIG_TILE=0: the 64/128-row tile)
_BIG_MOE = os.environ.get("BFLY_MOE_BIG_TILE", "1").strip().lower() not in ("0", "false", "no", "off")
# Host-side index checks of ops whose kernels cannot raise (BFLY_DEBUG_CHECKS; each costs a sync)
_DEBUG_CHECKS = os.environ.get("BFLY_DEBUG_CHECKS", "0").strip().lower() in ("1", "true", "yes", "on")


def set_poison(on: bool) -> None:
    """Allocate op outputs poisoned (debug / tests; costs one fill per output)."""
    global _POISON
    _POISON = bool(on)


def _poisoned(t: torch.Tensor) -> torch.Tensor:
    return t.fill_(float("nan") if t.is_floating_point() else -7777777)


def _empty(*shape, **kw) -> torch.Tensor:
    t = torch.empty(*shape, **kw)
    return _poisoned(t) if _POISON else t


def _empty_like(x: torch.Tensor, **kw) -> torch.Tensor:
    t = torch.empty_like(x, **kw)
    return _poisoned(t) if _POISON else t


_scope = threading.local()
_arena = _Arena()


def arena_scope(name) -> None:
    """Give this host thread its own workspace buffers (None: the process-wide set)."""
    _scope.name = name


def reserve_workspace(device, max_tokens: int, max_n: int, max_k: int, max_batch: int = 0,
                      max_ctx: int = 0, num_kv_heads: int = 0, head_dim: int = 128, shapes=()) -> None:
    """Pre-size every workspace for problems up to the given bounds (call before capture).
    `shapes`: the model's GEMM weight shapes (N, K); the split-K slab need is the max over them
    and every token-count bucket of the plan table (a tuned plan may split a small projection
    more than the largest one is split)."""
    if not load_library():
        return
    ws = 0
    nk = {(int(max_n), int(max_k))} | {(int(n), int(k)) for n, k in shapes}
    for m in sorted({1, 16, 32, 48, 64, 128, 256, 512, max_tokens}):
        if m > max_tokens:
            continue
        for n, k in nk:
            ws = max(ws, torch.ops.bfly.gemm_workspace_size(m, n, k))
    _arena.get(device, "gemm", ws // 4 + 1, torch.float32, zero=True)
    if max_batch and max_ctx:
        ns = max(torch.ops.bfly.attn_decode_splits(max_ctx, torch.ops.bfly.attn_decode_part_tokens(b, num_kv_heads, max_ctx))
                 for b in range(1, max_batch + 1))
        _arena.get(device, "attn_o", max_batch * num_kv_heads * ns * 16 * head_dim, torch.float32)
        _arena.get(device, "attn_ml", max_batch * num_kv_heads * ns * 16 * 2, torch.float32)
    _arena.get(device, "sample", max(max_batch, max_tokens, 1) * 64, torch.int64)
    _arena.get(device, "tkp", max(max_batch, max_tokens, 1) * 521, torch.float32)


# ---------------------------------------------------------------------------------------
# Ops
# ---------------------------------------------------------------------------------------
class Partial:
    """Output of a split-K GEMM whose reduce was deferred to its consumer (`linear(...,
    defer=True)`): `slabs` [sk, M, N] f32 live in the shared GEMM workspace and must be consumed
    (rms_norm / rope_kv fuse the reduce) or `materialize()`d before the next GEMM runs.
    `out` is the bf16 [M, N] buffer the result belongs in."""

    __slots__ = ("slabs", "out")

    def __init__(self, slabs: torch.Tensor, out: torch.Tensor):
        self.slabs, self.out = slabs, out

    @property
    def shape(self):
        return self.out.shape

    def materialize(self) -> torch.Tensor:
        torch.ops.bfly.splitk_reduce(self.slabs, self.out)
        return self.out


def materialize(x):
    return x.materialize() if isinstance(x, Partial) else x


class RowNormed:
    """RMSNorm output whose 1/rms row scale is left to the consuming GEMM (`rms_norm(...,
    rows=True)`, norm.hip rmsnorm_rows_kernel): `y` [M, dim] bf16 = x * w, `ssp` [M, chunks] f32
    partial sums of squares of x. `linear(RowNormed, ...)` scales row m of its result by
    rsqrt(sum(ssp[m]) / dim + eps) in the GEMM epilogue (before bias / SiLU / split-K slabs)."""

    __slots__ = ("y", "ssp", "eps")

    def __init__(self, y: torch.Tensor, ssp: torch.Tensor, eps: float):
        self.y, self.ssp, self.eps = y, ssp, eps

    @property
    def shape(self):
        return self.y.shape


_rowscale_ok: dict = {}


def rowscale_ok(M: int, N: int, K: int, epilogue: str = "none") -> bool:
    """True if the GEMM plan for this shape applies a RowScale (tile / decode-ring kernels)."""
    key = (M, N, K, epilogue)
    ok = _rowscale_ok.get(key)
    if ok is None:
        ok = load_library() and torch.ops.bfly.gemm_rowscale_check(M, N, K, EPILOGUES[epilogue]) == 0
        _rowscale_ok[key] = ok
    return ok


def rms_norm(x, w, eps: float, out=None, residual=None, rows: bool = False):
    """y = x * rsqrt(mean(x^2) + eps) * w; with `residual`: residual += x first (in place)
    and y is the norm of the updated residual (the fused add+norm of every block). `x` may be
    a deferred split-K GEMM output (`Partial`): its reduce is fused into this kernel.
    `rows=True` (GPU): return a `RowNormed` for a row-scaling consumer GEMM instead."""
    if rows and (isinstance(x, Partial) or _gpu(x)):
        src = x.slabs if isinstance(x, Partial) else x
        M, dim = src.shape[-2], src.shape[-1]
        if out is None:
            out = _empty(M, dim, dtype=w.dtype, device=w.device)
        ssp = _empty(M, torch.ops.bfly.rms_norm_rows_chunks(dim), dtype=torch.float32, device=w.device)
        torch.ops.bfly.rms_norm_rows(src, w, out, ssp, residual)
        return RowNormed(out, ssp, eps)
    if isinstance(x, Partial):
        if out is None:
            out = _empty_like(x.out)
        torch.ops.bfly.rms_norm_partial(x.slabs, w, eps, out, residual)
        return out
    if not _gpu(x):
        return ref.rms_norm(x, w, eps, out, residual)
    if out is None:
        out = _empty_like(x)
    torch.ops.bfly.rms_norm(x, w, eps, out, residual)
    return out


def rms_norm_route(x, w, eps: float, residual, router_w, top_k: int):
    """The fused add + RMSNorm of a MoE layer's FFN input that also routes the rows it
    normalises (norm.hip rmsnorm_partial_kernel<NV, E>): returns (y, (gates, topk_ids, topk_w))
    as `rms_norm` then `moe_route(y, router_w, top_k)` would, in one launch. Needs a deferred
    split-K input (`Partial`), a residual and 4 or 8 experts; otherwise returns (rms_norm(...),
    None) and the caller routes separately."""
    if (isinstance(x, Partial) and residual is not None
            and torch.ops.bfly.rms_norm_route_ok(router_w.shape[0], router_w.shape[1]) == 1):
        T = x.out.shape[0]
        E = router_w.shape[0]
        out = _empty_like(x.out)
        gates = _empty(T, E, dtype=torch.float32, device=out.device)
        ids = _empty(T, top_k, dtype=torch.int32, device=out.device)
        tw = _empty(T, top_k, dtype=torch.float32, device=out.device)
        torch.ops.bfly.rms_norm_partial_route(x.slabs, w, eps, out, residual, router_w, top_k, gates, ids, tw)
        return out, (gates, ids, tw)
    return rms_norm(x, w, eps, residual=residual), None


def layer_norm(x, w, b, eps: float, out=None, residual=None):
    if not _gpu(x):
        return ref.layer_norm(x, w, b, eps, out, residual)
    if out is None:
        out = _empty_like(x)
    torch.ops.bfly.layer_norm(x, w, b, eps, out, residual)
    return out


def rope_kv(qkv, positions, cos, sin, n_q: int, n_kv: int, slots=None, k_cache=None,
            v_cache=None):
    """In-place RoPE on the Q/K heads of a fused QKV row; optional paged KV append. Returns the
    (bf16) QKV rows; `qkv` may be a deferred split-K GEMM output whose reduce is fused here."""
    if isinstance(qkv, Partial):
        torch.ops.bfly.rope_kv(qkv.out, positions, cos, sin, n_q, n_kv, slots, k_cache, v_cache, qkv.slabs)
        return qkv.out
    if not _gpu(qkv):
        return ref.rope_kv(qkv, positions, cos, sin, n_q, n_kv, slots, k_cache, v_cache)
    torch.ops.bfly.rope_kv(qkv, positions, cos, sin, n_q, n_kv, slots, k_cache, v_cache)
    return qkv


def kv_append(k, v, slots, k_cache, v_cache):
    if not _gpu(k):
        return ref.kv_append(k, v, slots, k_cache, v_cache)
    torch.ops.bfly.kv_append(k, v, slots, k_cache, v_cache)


def silu_mul(gu, out=None, interleave: int = 0):
    if not _gpu(gu):
        return ref.silu_mul(gu, out, interleave)
    if out is None:
        out = _empty(*gu.shape[:-1], gu.shape[-1] // 2, dtype=gu.dtype, device=gu.device)
    torch.ops.bfly.silu_mul(gu, out, interleave)
    return out


def gelu(x, out=None):
    if not _gpu(x):
        return ref.gelu(x, out)
    if out is None:
        out = _empty_like(x)
    torch.ops.bfly.gelu(x, out)
    return out


def add(a, b, out=None):
    b = materialize(b)
    if not _gpu(a):
        return ref.add(a, b, out)
    if out is None:
        out = _empty_like(a)
    torch.ops.bfly.add(a, b, out)
    return out


def embed(ids, table, vstart: int = 0, out=None):
    if not _gpu(ids):
        return ref.embed(ids, table, vstart, out)
    if out is None:
        out = _empty(ids.numel(), table.shape[1], dtype=table.dtype, device=table.device)
    torch.ops.bfly.embed(ids, table, out, vstart)
    return out


def gather_rows(src, idx, out=None):
    """out[i] = src[idx[i]] (rows of a 2-D tensor; `idx` int32 / int64). Rows whose idx is < 0
    keep what `out` holds (pass a pre-filled `out`). Our row-gather kernel on the GPU, not
    torch's index_select (elementwise.hip gather_rows_kernel)."""
    if out is None:
        out = _empty(idx.numel(), *src.shape[1:], dtype=src.dtype, device=src.device)
    if not _gpu(src):
        return ref.gather_rows(src, idx, out)
    s2 = src if src.dim() == 2 else src.view(src.shape[0], -1)
    o2 = out if out.dim() == 2 else out.view(out.shape[0], -1)
    if _DEBUG_CHECKS and not torch.cuda.is_current_stream_capturing() and idx.numel():
        hi = int(idx.max())
        if hi >= src.shape[0]:
            raise IndexError(f"gather_rows: index {hi} out of range for {src.shape[0]} source rows")
    torch.ops.bfly.gather_rows(s2, idx, o2)
    return out


def sample_pack(scores, ids):
    """Per-shard sampling winners -> [rows, 2] f32 (score, id) pairs for the TP all-gather."""
    if not _gpu(scores):
        return ref.sample_pack(scores, ids)
    pair = _empty(scores.numel(), 2, dtype=torch.float32, device=scores.device)
    torch.ops.bfly.sample_pack(scores.contiguous(), ids.contiguous(), pair)
    return pair


def sample_merge(allp):
    """All-gathered pairs [tp, rows, 2] -> int32 ids of the best score per row (lowest rank on
    ties: torch.argmax's first maximum)."""
    if not _gpu(allp):
        return ref.sample_merge(allp)
    out = _empty(allp.shape[1], dtype=torch.int32, device=allp.device)
    torch.ops.bfly.sample_merge(allp.contiguous(), out)
    return out


def sample(logits, temps=None, seeds=None, vstart: int = 0, out_ids=None, out_scores=None, thresh=None,
           check_finite: bool = False):
    """Greedy / Gumbel-max sampling over a (vocab-shard of) logits -> (ids int32, scores f32).
    `thresh` [rows] f32: per-row lower bound on logit / temperature (top-k / top-p filter).
    `check_finite`: rows with an Inf / NaN logit get id -1 and score +inf (the NaN guard)."""
    if not _gpu(logits):
        return ref.sample(logits, temps, seeds, vstart, thresh, check_finite)
    rows = logits.shape[0]
    if out_ids is None:
        out_ids = _empty(rows, dtype=torch.int32, device=logits.device)
    if out_scores is None:
        out_scores = _empty(rows, dtype=torch.float32, device=logits.device)
    ws = _arena.get(logits.device, "sample", rows * 64, torch.int64)
    torch.ops.bfly.sample(logits, temps, seeds, vstart, out_ids, out_scores, ws, thresh, check_finite)
    return out_ids, out_scores


def topkp_threshold(logits, temps, top_k, top_p, reduce_sum=None, reduce_max=None,
                    use_k: bool = True, use_p: bool = True):
    """Exact per-row top-k / top-p threshold on logit / temperature by radix select (4 passes
    of 8 bits per filter, sample.hip tkp_*). `reduce_sum(t)` / `reduce_max(t)`: in-place
    all-reduces over the TP group applied to every histogram / the row maxima, so vocab shards
    select together (None: unsharded). `use_k` / `use_p`: skip a filter no row uses. Returns
    thresh [R] f32 (-inf = unfiltered row), the `thresh` argument of `sample`."""
    if not _gpu(logits):
        return ref.topkp_threshold(logits, temps, top_k, top_p, reduce_sum, reduce_max, use_k, use_p)
    R = logits.shape[0]
    L = torch.ops.bfly
    ws = _arena.get(logits.device, "tkp", R * 521, torch.float32)[: R * 521]
    zero_(ws)
    # the row-max slot starts at the smallest ordered key (INT_MIN = below signed_ordered(-inf)):
    # a zero would read as +0.0 and clamp the max of an all-negative row
    L.fill32_(ws[R * 8:R * 9], -2 ** 31)
    L.tkp_begin(logits, temps, top_k, top_p, ws)
    if reduce_max is not None:
        reduce_max(ws[R * 8:R * 9].view(torch.int32))
    hist = ws[R * 9:].view(R, 512)
    for phase, on in ((0, use_k), (1, use_p)):
        if not on:
            continue
        for p in range(4):
            L.tkp_pass(logits, temps, ws, p, phase)
            if reduce_sum is not None:
                reduce_sum(hist)
            L.tkp_select(top_p, ws, R, p, phase)
    thr = _empty(R, dtype=torch.float32, device=logits.device)
    L.tkp_final(ws, R, thr)
    return thr


def pack_w256(w: torch.Tensor) -> torch.Tensor:
    """A [N, K] weight in the K-tile-blocked layout [N/256][K/64][256][64] (returned viewed as
    [N, K]) that the packed decode GEMM reads (gemm.hip launch_gemm_packed)."""
    N, K = w.shape
    return w.view(N // 256, 256, K // 64, 64).permute(0, 2, 1, 3).contiguous().view(N, K)


def linear(x, w, bias=None, epilogue: str = "none", out=None, defer: bool = False, packed=None):
    """y = x @ w.T (+ bias) with optional fused SwiGLU epilogue ('silu': w rows gate/up
    interleaved in 16-row groups, output width w.shape[0] // 2). `defer=True` (no bias /
    epilogue): when the plan splits K, return a `Partial` whose reduce the consumer fuses.
    `packed`: the weight's pack_w256 copy: used when the shape's plan has a packed form (decode
    tile plans), else `w`."""
    rn = None
    if isinstance(x, RowNormed):   # consumer of a row-split RMSNorm: the GEMM applies 1/rms
        rn, x = x, x.y
    if not _gpu(x):
        return ref.linear(x, w, bias, epilogue, out)
    if packed is not None and bias is None and epilogue in ("none", "silu") and not (defer and epilogue != "none"):
        M, N = x.shape[0], w.shape[0]
        if out is None:
            out = _empty(M, N // 2 if epilogue == "silu" else N, dtype=x.dtype, device=x.device)
        need = torch.ops.bfly.gemm_workspace_size(M, N, x.shape[1])
        ws = _arena.get(x.device, "gemm", need // 4 + 1, torch.float32, zero=True) if need else None
        sk = torch.ops.bfly.gemm_packed(x, packed, out, EPILOGUES[epilogue], rn.ssp if rn is not None else None,
                                        rn.eps if rn is not None else 0.0, None, 0, 1, ws, bool(defer))
        if sk == 1:
            return out
        if sk > 1:     # deferred split-K slabs for the consumer
            off = torch.ops.bfly.gemm_slab_offset()
            return Partial(ws[off:off + sk * M * N].view(sk, M, N), out)
    if defer and bias is None and epilogue == "none":
        M, N = x.shape[0], w.shape[0]
        if out is None:
            out = _empty(M, N, dtype=x.dtype, device=x.device)
        need = torch.ops.bfly.gemm_workspace_size(M, N, x.shape[1])
        ws = _arena.get(x.device, "gemm", need // 4 + 1, torch.float32, zero=True)
        if rn is not None:
            sk = torch.ops.bfly.gemm_deferred_rs(x, w, out, ws, rn.ssp, rn.eps)
        else:
            sk = torch.ops.bfly.gemm_deferred(x, w, out, ws)
        if sk == 1:
            return out
        off = torch.ops.bfly.gemm_slab_offset()
        return Partial(ws[off:off + sk * M * N].view(sk, M, N), out)
    epi = EPILOGUES["bias"] if (bias is not None and epilogue == "none") else EPILOGUES[epilogue]
    if epilogue == "silu" and bias is not None:
        raise ValueError("bias + silu epilogue not supported")
    M, N = x.shape[0], w.shape[0]
    nout = N // 2 if epilogue == "silu" else N
    if out is None:
        out = _empty(M, nout, dtype=x.dtype, device=x.device)
    need = torch.ops.bfly.gemm_workspace_size(M, N, x.shape[1])
    # zero-initialised once: its head holds the split-K arrival counters, which every GEMM
    # leaves re-armed at zero
    ws = _arena.get(x.device, "gemm", need // 4 + 1, torch.float32, zero=True) if need else None
    if rn is not None:
        torch.ops.bfly.gemm_rs(x, w, out, bias, epi, ws, rn.ssp, rn.eps)
    else:
        torch.ops.bfly.gemm(x, w, out, bias, epi, ws)
    return out


def linear_silu_gate(x, w, gates, e0: int, num_local: int, packed=None):
    """The dense MoE decode gate/up GEMM over the concatenated local experts: SwiGLU, then every
    expert's column block scaled by its routing weight gates[:, e0 + e] — `linear(x, w, 'silu')`
    followed by `moe_gate_scale_`, bit for bit, in one launch (the tile kernel's epilogue).
    `packed`: the weight's pack_w256 copy (used when the plan has a packed form)."""
    if isinstance(x, RowNormed) or not _gpu(x):
        h = linear(x, w, epilogue="silu")
        return moe_gate_scale_(h, gates, e0, num_local)
    out = _empty(x.shape[0], w.shape[0] // 2, dtype=x.dtype, device=x.device)
    if packed is not None and torch.ops.bfly.gemm_packed(x, packed, out, 3, None, 0.0, gates, e0, num_local) > 0:
        return out
    torch.ops.bfly.gemm_silu_gate(x, w, out, gates, e0, num_local)
    return out


def gemm_plan(M: int, N: int, K: int) -> dict:
    load_library()
    k, mt, nt, bm, bn, sk, wk = torch.ops.bfly.gemm_plan(M, N, K)
    return {"kind": ("skinny", "tile", "big", "dec", "big8", "mid8", "big4", "mid4")[k], "mt": mt, "nt": nt, "wk": wk, "bm": bm, "bn": bn,
            "splitk": sk}


def attn_prefill(q, k, v, cu_seqlens, max_seqlen: int, scale: float, causal: bool = True,
                 out=None, cu_seqlens_k=None, return_lse: bool = False):
    """Varlen flash attention (K3). `cu_seqlens_k`: keys of each sequence come from other
    rows than its queries (non-causal; context-parallel ring steps). `return_lse`: also return
    the per-(row, head) natural-log sum-exp of the scaled scores [T, Hq] f32 (-inf: no keys),
    which `attn_lse_merge_` uses to combine attention over key chunks."""
    if not _gpu(q):
        return ref.attn_prefill(q, k, v, cu_seqlens, max_seqlen, scale, causal, out, cu_seqlens_k, return_lse)
    if out is None:
        out = _empty(q.shape, dtype=q.dtype, device=q.device)
    lse = _empty(q.shape[0], q.shape[1], dtype=torch.float32, device=q.device) if return_lse else None
    torch.ops.bfly.attn_prefill(q, k, v, cu_seqlens, max_seqlen, scale, causal, out, cu_seqlens_k, lse)
    return (out, lse) if return_lse else out


def attn_prefill_paged(q, k_cache, v_cache, tables, cu_q, positions, max_q: int, scale: float, out=None):
    """Chunked prefill attention over the paged cache (attention_paged.hip): query rows
    [cu_q[s], cu_q[s+1]) of sequence s at `positions` attend causally to the sequence's cached
    keys through tables[s] — the cached prefix and the chunk itself (already appended by
    rope_kv) in one pass, no gather, no log-sum-exp merge. Caches bf16 or FP8."""
    if not _gpu(q):
        return ref.attn_prefill_paged(q, k_cache, v_cache, tables, cu_q, positions, max_q, scale, out)
    if out is None:
        out = _empty(q.shape, dtype=q.dtype, device=q.device)
    torch.ops.bfly.attn_prefill_paged(q, k_cache, v_cache, tables, cu_q, positions, int(max_q), float(scale), out)
    return out


def attn_lse_merge_(acc_o, acc_lse, o, lse):
    """K16: fold a partial attention result (o bf16 [T, H, D], lse [T, H]) into running f32
    accumulators (acc_o [T, H, D], acc_lse [T, H]) in place."""
    if not _gpu(acc_o):
        return ref.attn_lse_merge_(acc_o, acc_lse, o, lse)
    torch.ops.bfly.attn_lse_merge(acc_o, acc_lse, o, lse)
    return acc_o, acc_lse


def attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale: float, max_ctx: int,
                part_tokens: int = DECODE_PART_TOKENS, out=None):
    """One query token per sequence against the paged cache. `max_ctx` bounds ctx_lens (it
    fixes the split-KV grid, so it is a static parameter under graph capture)."""
    if not _gpu(q):
        return ref.attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale, max_ctx,
                               part_tokens, out)
    B, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    if out is None:
        out = _empty(B, Hq, D, dtype=q.dtype, device=q.device)
    if part_tokens <= 0:
        part_tokens = torch.ops.bfly.attn_decode_part_tokens(B, Hkv, max_ctx)
    ns = torch.ops.bfly.attn_decode_splits(max_ctx, part_tokens)
    po = pml = None
    if ns > 1:
        po = _arena.get(q.device, "attn_o", B * Hkv * ns * 16 * D, torch.float32)
        pml = _arena.get(q.device, "attn_ml", B * Hkv * ns * 16 * 2, torch.float32)
    torch.ops.bfly.attn_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale, max_ctx,
                               part_tokens, out, po, pml)
    return out


def init_hash_(out, grow0: int, gcol0: int, gcols: int, seed: int, amp: float):
    """Fill a 2-D (view of a) weight shard with partition-independent hashed uniform values."""
    if not _gpu(out):
        return ref.init_hash(out, grow0, gcol0, gcols, seed, amp)
    torch.ops.bfly.init_hash(out, grow0, gcol0, gcols, seed & 0xFFFFFFFF, amp)
    return out


def moe_route(x, wr, top_k: int, gates=None, topk_ids=None, topk_w=None):
    if not _gpu(x):
        return ref.moe_route(x, wr, top_k)
    T, E = x.shape[0], wr.shape[0]
    if gates is None:
        gates = _empty(T, E, dtype=torch.float32, device=x.device)
    if topk_ids is None:
        topk_ids = _empty(T, top_k, dtype=torch.int32, device=x.device)
    if topk_w is None:
        topk_w = _empty(T, top_k, dtype=torch.float32, device=x.device)
    torch.ops.bfly.moe_route(x, wr, top_k, gates, topk_ids, topk_w)
    return gates, topk_ids, topk_w


def moe_sparse_ffn(x, topk_ids, topk_w, gu_w, down_w, e0: int, num_local: int, ffn: int,
                   expected_slots: Optional[int] = None, block_counts: Optional[tuple] = None):
    """Routed expert FFN: permute the (token, k) pairs of the local experts into per-expert
    row slots (moe_align), grouped gate/up GEMM with fused SiLU over gathered token rows,
    grouped down GEMM, weighted combine back to token order. Only routed rows are computed
    (the dense path computes every local expert for every token).
    `block_counts` = (counts [nblk] int32 on the device, cap): the rows are nblk blocks of `cap`
    rows of which only the first counts[b] are valid (the EP IPC prefill receive buffer, sized
    for the worst case): the other rows get no expert work and no output row."""
    if not _gpu(x):
        if block_counts is not None:
            cnt, cap = block_counts
            r = torch.arange(x.shape[0]) % cap
            ok = r < cnt.cpu().long()[torch.arange(x.shape[0]) // cap]
            topk_ids = topk_ids.masked_fill(~ok.unsqueeze(1), -1)
        return ref.moe_sparse_ffn(x, topk_ids, topk_w, gu_w, down_w, e0, num_local, ffn)
    T, H = x.shape
    k = topk_ids.shape[1]
    TK = T * k
    if TK == 0:
        return zero_(torch.empty(T, H, dtype=x.dtype, device=x.device))
    L = torch.ops.bfly
    dev = x.device
    bcnt, bcap = block_counts if block_counts is not None else (None, 0)
    # tile rows from the expected rows per expert (all slots are local in the EP dispatch):
    # one 128-row tile reads each expert's weights once where two 64-row tiles would twice
    # `expected_slots`: (token, k) pairs expected to be local (the EP dispatch pads with
    # non-local / empty slots; they cost nothing but must not size the launch)
    exp = TK if expected_slots is None else max(1, min(TK, expected_slots))
    # prefill-scale expert batches (>= 256 rows per local expert on average): the 8-phase
    # 256x256 tile over the tile list (gemm.hip gemm_big8_kernel<GROUPED>)
    bm = 256 if (exp >= 256 * num_local and H % 256 == 0 and (2 * ffn) % 256 == 0 and _BIG_MOE) else \
        (128 if exp >= 96 * num_local else 64)
    rows = _arena.get(dev, "moe_rows", TK, torch.int32)[:TK]
    slot_of = _arena.get(dev, "moe_slot", TK, torch.int32)[:TK]
    nt = L.moe_max_tiles(TK, num_local, bm)
    tiles = _arena.get(dev, "moe_tiles", nt * 4, torch.int32)[:nt * 4].view(nt, 4)
    count = _arena.get(dev, "moe_count", 1, torch.int32)[:1]
    L.moe_align(topk_ids, e0, num_local, rows, slot_of, tiles, count, bm, bcnt, bcap)
    hmid = _empty(TK, ffn, dtype=x.dtype, device=dev)
    L.moe_grouped_gemm(x, gu_w, hmid, rows, tiles, count, 2 * ffn * H, 2 * ffn, H, num_local, EPILOGUES["silu"], bm)
    out = _empty(T, H, dtype=x.dtype, device=dev)
    sk = moe_down_splits(exp, num_local, H, ffn, bm)
    if sk > 1:
        # decode-sized expert batches: split K of the down projection over sk workgroups so the
        # chip fills; the slab reduce is folded into the weighted combine
        part = _arena.get(dev, "moe_part", sk * TK * H, torch.float32)[: sk * TK * H].view(sk, TK, H)
        L.moe_grouped_gemm(hmid, down_w, hmid.new_empty(TK, H), None, tiles, count, ffn, H, ffn, num_local,
                           EPILOGUES["none"], bm, part)
        L.moe_combine_slabs(part, slot_of, topk_w, out, bcnt, bcap)
        return out
    y = _empty(TK, H, dtype=x.dtype, device=dev)
    L.moe_grouped_gemm(hmid, down_w, y, None, tiles, count, ffn, H, ffn, num_local, EPILOGUES["none"], bm)
    L.moe_combine(y, slot_of, topk_w, out, bcnt, bcap)
    return out


def ep_pack(x, ids, w, slots, experts_per_rank: int, ep: int, cap: int):
    """Pack a fixed-capacity EP dispatch (see ops.reference.ep_pack for the layout)."""
    if not _gpu(x):
        return ref.ep_pack(x, ids, w, slots, experts_per_rank, ep, cap)
    T, H = x.shape
    k = ids.shape[1]
    send = _empty(ep * cap, H, dtype=x.dtype, device=x.device)
    meta = _empty(ep * cap, 2 * k, dtype=torch.float32, device=x.device)
    slot = _empty(T, ep, dtype=torch.int32, device=x.device)
    torch.ops.bfly.ep_pack(x.contiguous(), ids.contiguous(), w.contiguous(), slots, experts_per_rank, ep, cap,
                           send, meta, slot)
    return send, meta, slot


def ep_combine(back, slot):
    """Sum each token's returned partial outputs (one per rank it was sent to)."""
    if not _gpu(back):
        return ref.ep_combine(back, slot)
    out = _empty(slot.shape[0], back.shape[1], dtype=back.dtype, device=back.device)
    torch.ops.bfly.ep_combine(back, slot, out)
    return out


def moe_down_splits(TK: int, num_local: int, H: int, ffn: int, bm: int, cus: int = 256) -> int:
    """Split-K factor of the grouped down projection: enough workgroups for ~2 per CU, with
    at least 16 K-tiles (1024 columns) per split (none for the 256-row big tile)."""
    if bm == 256:
        return 1
    tiles = -(-TK // bm) + (num_local if TK >= num_local else 0)
    wgs = max(1, tiles) * (H // 128)
    sk = 1
    while wgs * sk * 2 <= 2 * cus and (ffn // 64) // (sk * 2) >= 16 and sk < 8:
        sk *= 2
    return sk


def moe_gate_scale_(h, gates, e0: int, num_local: int):
    if not _gpu(h):
        return ref.moe_gate_scale(h, gates, e0, num_local)
    torch.ops.bfly.moe_gate_scale(h, gates, e0, num_local)
    return h
