"""Decoder-only transformer LM covering the Llama-3, Mixtral and GPT-2 families.

One class, arch-specific switches from ModelConfig (norm, position embedding, MLP kind,
biases, MoE). The model holds only its shard (models/shard.py) and runs one pipeline stage:

  first stage : token (+ learned position) embedding, vocab-parallel (TP all-reduce)
  every layer : norm -> fused QKV GEMM -> RoPE + paged-KV append -> attention
                (flash prefill / paged decode) -> O GEMM -> TP all-reduce ->
                fused residual-add + norm -> FFN (SwiGLU with the activation fused into the
                gate/up GEMM epilogue | GELU MLP | dense-dispatch MoE) -> TP all-reduce
  last stage  : final norm on the rows that need logits -> vocab-parallel LM head

Sequence parallelism (BFLY_SEQ_PARALLEL, TP prefill steps, `_forward_sp`): the residual
stream lives split by tokens over the TP group; each all-reduce becomes a reduce-scatter
(into the rank's token shard, where the residual add + norm run on 1/tp of the rows) and an
all-gather of the normed activations feeding the next column-parallel GEMM. Same link bytes
as the all-reduce; norm work and residual memory drop by tp (SURVEY.md §2.6 SP).

The residual stream is carried as (residual, pending delta): each block's "add + norm" is
ONE kernel (rms_norm with residual=...), so the residual add never costs its own pass.

Weights live in fused local tensors (qkv, interleaved gate/up, stacked experts). The
checkpoint and the random initialiser work on *logical* parameters (HF-style names, global
shapes, shard slices) through `logical_params()`, which is what makes a checkpoint written
under one partition plan loadable under another.
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass
from typing import Callable, Optional

import torch

from .. import ops
from ..utils import flags
from ..config import ModelConfig
from ..engine.batch import ForwardBatch
from ..parallel.comm import Communicator
from .shard import LocalDims, Shard, local_dims

G16 = ops.SILU_INTERLEAVE


@dataclass
class LogicalParam:
    name: str
    global_shape: tuple
    split_dim: Optional[int]      # dim along which the local piece is a contiguous slice
    offset: int                   # start of the local piece along split_dim
    length: int                   # extent of the local piece along split_dim
    init: str                     # "normal" | "ones" | "zeros"
    get: Callable[[], torch.Tensor]
    set: Callable[[torch.Tensor], None]
    owner: bool = True            # canonical writer of this slice (replicas dedupe on save)

    def local_shape(self) -> tuple:
        s = list(self.global_shape)
        if self.split_dim is not None:
            s[self.split_dim] = self.length
        return tuple(s)


def _name_seed(name: str, seed: int) -> int:
    return (zlib.crc32(name.encode()) ^ (seed * 0x9E3779B1)) & 0xFFFFFFFF


class TransformerLM:
    def __init__(self, cfg: ModelConfig, shard: Shard = Shard(), device="cpu",
                 dtype: torch.dtype = torch.bfloat16, comm: Optional[Communicator] = None):
        self.cfg = cfg
        self.shard = shard
        self.device = torch.device(device)
        self.dtype = dtype
        self.comm = comm or Communicator.single()
        self.dims: LocalDims = local_dims(cfg, shard)
        self.layer_ids = list(shard.layers(cfg))
        self.first = shard.is_first(cfg)
        self.last = shard.is_last(cfg)
        self.tp = shard.tp_size
        self.ep = shard.ep_size
        # fuse split-K GEMM reduces into the consuming kernels: QKV -> rope_kv always (no
        # collective in between), O / down -> add+rmsnorm when no TP all-reduce sits between
        defer = self.device.type == "cuda" and flags.get("BFLY_DEFER_REDUCE")
        self.defer_qkv = defer and cfg.pos_emb == "rope"
        # (tp > 1: the IPC all-reduce takes the split-K slabs and reduces them in its publish)
        self.defer_reduce = defer and cfg.norm == "rms" and (
            self.tp == 1 or getattr(self.comm, "custom_ar", None) is not None)
        # decode add+RMSNorm split over (row, column-chunk) workgroups with the 1/rms row scale
        # applied by the consuming QKV / gate-up GEMM (ops.RowNormed); tp == 1 only (with TP the
        # IPC all-reduce fuses the norm), dense FFNs (the MoE router reads the normed rows too)
        self.rowscale_rows = (flags.get("BFLY_NORM_ROWSCALE_MAX_ROWS")
                              if (self.device.type == "cuda" and cfg.norm == "rms" and self.tp == 1
                                  and not cfg.is_moe and flags.get("BFLY_NORM_ROWSCALE")) else 0)
        if self.device.type == "cuda" and cfg.head_dim != 128:
            raise NotImplementedError(f"GPU attention kernels need head_dim 128 (got {cfg.head_dim})")
        self.p: dict[str, torch.Tensor] = {}
        # K-tile-blocked copies of the gate/up weights for the decode GEMMs (pack_decode_weights)
        self.packed: dict[str, torch.Tensor] = {}
        self._alloc()
        self.cos = self.sin = None
        if cfg.pos_emb == "rope":
            self.cos, self.sin = ops.rope_tables(cfg.head_dim, cfg.max_position, cfg.rope_theta,
                                                 cfg.rope_scaling, device=self.device)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.seq_parallel = self.tp > 1 and self.ep == 1 and flags.get("BFLY_SEQ_PARALLEL")
        self.sp_min_tokens = flags.get("BFLY_SEQ_PARALLEL_MIN_TOKENS")

    # ------------------------------------------------------------------------------------
    # parameters
    # ------------------------------------------------------------------------------------
    def _alloc(self):
        c, d = self.cfg, self.dims
        h, D = c.hidden_size, c.head_dim
        z = lambda *s: torch.zeros(*s, dtype=self.dtype, device=self.device)  # noqa: E731
        norm_b = c.norm == "layer"
        if self.first:
            self.p["embed"] = z(d.vocab, h)
            if c.pos_emb == "learned":
                self.p["pos_embed"] = z(c.max_position, h)
        for i in self.layer_ids:
            pre = f"l{i}."
            self.p[pre + "in_w"] = z(h)
            if norm_b:
                self.p[pre + "in_b"] = z(h)
            self.p[pre + "qkv_w"] = z((d.hq + 2 * d.hkv) * D, h)
            self.p[pre + "o_w"] = z(h, d.hq * D)
            if c.bias:
                self.p[pre + "qkv_b"] = z((d.hq + 2 * d.hkv) * D)
                self.p[pre + "o_b"] = z(h)
            self.p[pre + "post_w"] = z(h)
            if norm_b:
                self.p[pre + "post_b"] = z(h)
            if c.is_moe:
                self.p[pre + "router_w"] = z(c.num_experts, h)
                self.p[pre + "moe_gu_w"] = z(d.experts * 2 * d.ffn, h)
                self.p[pre + "moe_down_w"] = z(h, d.experts * d.ffn)
            elif c.act == "silu":
                self.p[pre + "gu_w"] = z(2 * d.ffn, h)
                self.p[pre + "down_w"] = z(h, d.ffn)
            else:
                self.p[pre + "fc_w"] = z(d.ffn, h)
                self.p[pre + "proj_w"] = z(h, d.ffn)
                if c.bias:
                    self.p[pre + "fc_b"] = z(d.ffn)
                    self.p[pre + "proj_b"] = z(h)
        if self.last:
            self.p["final_w"] = z(h)
            if norm_b:
                self.p["final_b"] = z(h)
            if not c.tie_embeddings:
                self.p["head"] = z(d.vocab, h)
            elif not self.first:
                # tied head on a last stage that does not hold the embedding: its own copy
                self.p["head"] = z(d.vocab, h)

    # decode projections in the order their packed copies are made when HBM is short: gate/up
    # first (the largest decode GEMM), then the others
    _PACK_ORDER = ("gu_w", "moe_gu_w", "qkv_w", "o_w", "down_w", "moe_down_w")

    _PACK_EPI = {"gu_w": 2, "moe_gu_w": 3}    # GEMM epilogue of each kind (others: none)

    def _packable(self) -> list:
        """Weights whose decode GEMM has a packed-weight plan at some batch of 1-256 rows."""
        if self.device.type != "cuda" or not ops.load_library():
            return []
        names = []
        for kind in self._PACK_ORDER:
            for i in self.layer_ids:
                k = f"l{i}.{kind}"
                w = self.p.get(k)
                if (w is not None and w.shape[0] % 256 == 0 and w.shape[1] % 64 == 0
                        and any(torch.ops.bfly.gemm_packed_check(m, w.shape[0], w.shape[1], self._PACK_EPI.get(kind, 0)) == 0
                                for m in (1, 16, 64, 128, 256, 512))):
                    names.append(k)
        return names

    def packed_decode_bytes(self, kinds=None) -> int:
        """HBM a pack_decode_weights(kinds) call would add."""
        return sum(self.p[k].numel() * self.p[k].element_size() for k in self._packable()
                   if kinds is None or k.split(".", 1)[1] in kinds)

    def pack_decode_weights(self, budget_bytes: Optional[int] = None, kinds=None) -> int:
        """Keep K-tile-blocked copies (ops.pack_w256) of the decode projections' weights, read by
        the decode GEMMs whose plan is a 16 / 32 / 64-row tile or a mid-M kernel (batches of 1-512
        rows): each weight stage is
        one contiguous run of memory instead of a row segment per weight row, 8 % faster on the
        Llama-3-70B gate/up GEMM with bitwise the same result (tools/packed_probe.py). Whole
        projection kinds, in the order of `kinds` (None: _PACK_ORDER), while they fit
        `budget_bytes` (None: all). The engine
        calls it once, after the weights are final; weights must not change afterwards. Returns
        the bytes added."""
        if self.device.type != "cuda":
            return 0
        added = 0
        for kind in (self._PACK_ORDER if kinds is None else kinds):
            names = [k for k in self._packable() if k.split(".", 1)[1] == kind]
            size = sum(self.p[k].numel() * self.p[k].element_size() for k in names)
            if not names or (budget_bytes is not None and added + size > budget_bytes):
                continue
            for k in names:
                self.packed[k] = ops.pack_w256(self.p[k])
            added += size
        return added

    @property
    def head_weight(self) -> torch.Tensor:
        return self.p["head"] if "head" in self.p else self.p["embed"]

    def local_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.p.values())

    def logical_params(self) -> list[LogicalParam]:
        """Every logical (HF-style) parameter slice this rank holds."""
        c, d, s = self.cfg, self.dims, self.shard
        h, D = c.hidden_size, c.head_dim
        tp0 = s.tp_rank == 0
        ep0 = s.ep_rank == 0
        out: list[LogicalParam] = []

        def rows(t, a, n):
            return (lambda: t[a:a + n]), (lambda x: t[a:a + n].copy_(x))

        def whole(t):
            return (lambda: t), (lambda x: t.copy_(x.view(t.shape)))

        def add(name, gshape, split, off, length, init, getset, owner=True):
            out.append(LogicalParam(name, tuple(gshape), split, off, length, init, getset[0], getset[1], owner))

        norm_b = c.norm == "layer"
        vlen = max(0, min(c.vocab_size, d.vocab0 + d.vocab) - d.vocab0)
        if self.first:
            add("embed_tokens.weight", (c.vocab_size, h), 0, d.vocab0, vlen, "normal",
                rows(self.p["embed"], 0, vlen), owner=ep0)
            if c.pos_emb == "learned":
                add("pos_embed.weight", (c.max_position, h), None, 0, 0, "normal",
                    whole(self.p["pos_embed"]), owner=tp0 and ep0)
        kv_rep = max(1, self.tp // c.num_kv_heads)            # tp ranks sharing one kv head
        kv_owner = (s.tp_rank % kv_rep == 0) and ep0
        for i in self.layer_ids:
            pre, L = f"l{i}.", f"layers.{i}."
            add(L + "input_norm.weight", (h,), None, 0, 0, "ones", whole(self.p[pre + "in_w"]), tp0 and ep0)
            if norm_b:
                add(L + "input_norm.bias", (h,), None, 0, 0, "zeros", whole(self.p[pre + "in_b"]), tp0 and ep0)
            qkv = self.p[pre + "qkv_w"]
            nq, nkv = d.hq * D, d.hkv * D
            add(L + "attn.q_proj.weight", (c.q_size, h), 0, d.q_head0 * D, nq, "normal", rows(qkv, 0, nq), ep0)
            add(L + "attn.k_proj.weight", (c.kv_size, h), 0, d.kv_head0 * D, nkv, "normal", rows(qkv, nq, nkv), kv_owner)
            add(L + "attn.v_proj.weight", (c.kv_size, h), 0, d.kv_head0 * D, nkv, "normal", rows(qkv, nq + nkv, nkv), kv_owner)
            if c.bias:
                qb = self.p[pre + "qkv_b"]
                add(L + "attn.q_proj.bias", (c.q_size,), 0, d.q_head0 * D, nq, "normal", rows(qb, 0, nq), ep0)
                add(L + "attn.k_proj.bias", (c.kv_size,), 0, d.kv_head0 * D, nkv, "normal", rows(qb, nq, nkv), kv_owner)
                add(L + "attn.v_proj.bias", (c.kv_size,), 0, d.kv_head0 * D, nkv, "normal", rows(qb, nq + nkv, nkv), kv_owner)
            ow = self.p[pre + "o_w"]
            add(L + "attn.o_proj.weight", (h, c.q_size), 1, d.q_head0 * D, nq, "normal", whole(ow), ep0)
            if c.bias:
                add(L + "attn.o_proj.bias", (h,), None, 0, 0, "normal", whole(self.p[pre + "o_b"]), tp0 and ep0)
            add(L + "post_norm.weight", (h,), None, 0, 0, "ones", whole(self.p[pre + "post_w"]), tp0 and ep0)
            if norm_b:
                add(L + "post_norm.bias", (h,), None, 0, 0, "zeros", whole(self.p[pre + "post_b"]), tp0 and ep0)
            F, Fg = d.ffn, c.intermediate_size
            if c.is_moe:
                add(L + "moe.router.weight", (c.num_experts, h), None, 0, 0, "normal",
                    whole(self.p[pre + "router_w"]), tp0 and ep0)
                gu, dn = self.p[pre + "moe_gu_w"], self.p[pre + "moe_down_w"]
                for el in range(d.experts):
                    e = d.expert0 + el
                    E = L + f"moe.experts.{e}."
                    blk = gu[el * 2 * F:(el + 1) * 2 * F]
                    add(E + "gate_proj.weight", (Fg, h), 0, d.ffn0, F, "normal", self._gu_getset(blk, 0), True)
                    add(E + "up_proj.weight", (Fg, h), 0, d.ffn0, F, "normal", self._gu_getset(blk, 1), True)
                    dcols = dn[:, el * F:(el + 1) * F]
                    add(E + "down_proj.weight", (h, Fg), 1, d.ffn0, F, "normal",
                        ((lambda t=dcols: t), (lambda x, t=dcols: t.copy_(x))), True)
            elif c.act == "silu":
                gu = self.p[pre + "gu_w"]
                add(L + "mlp.gate_proj.weight", (Fg, h), 0, d.ffn0, F, "normal", self._gu_getset(gu, 0), ep0)
                add(L + "mlp.up_proj.weight", (Fg, h), 0, d.ffn0, F, "normal", self._gu_getset(gu, 1), ep0)
                add(L + "mlp.down_proj.weight", (h, Fg), 1, d.ffn0, F, "normal", whole(self.p[pre + "down_w"]), ep0)
            else:
                add(L + "mlp.fc.weight", (Fg, h), 0, d.ffn0, F, "normal", whole(self.p[pre + "fc_w"]), ep0)
                add(L + "mlp.proj.weight", (h, Fg), 1, d.ffn0, F, "normal", whole(self.p[pre + "proj_w"]), ep0)
                if c.bias:
                    add(L + "mlp.fc.bias", (Fg,), 0, d.ffn0, F, "normal", whole(self.p[pre + "fc_b"]), ep0)
                    add(L + "mlp.proj.bias", (h,), None, 0, 0, "normal", whole(self.p[pre + "proj_b"]), tp0 and ep0)
        if self.last:
            add("final_norm.weight", (h,), None, 0, 0, "ones", whole(self.p["final_w"]), tp0 and ep0)
            if norm_b:
                add("final_norm.bias", (h,), None, 0, 0, "zeros", whole(self.p["final_b"]), tp0 and ep0)
            if not c.tie_embeddings:
                add("lm_head.weight", (c.vocab_size, h), 0, d.vocab0, vlen, "normal",
                    rows(self.p["head"], 0, vlen), ep0)
            elif "head" in self.p:
                # tied copy on a stage without the embedding: same logical tensor, not an owner
                add("embed_tokens.weight", (c.vocab_size, h), 0, d.vocab0, vlen, "normal",
                    rows(self.p["head"], 0, vlen), owner=False)
        return out

    @staticmethod
    def _gu_getset(gu: torch.Tensor, which: int):
        """Access the gate (0) or up (1) rows of a 16-row interleaved [2F, h] block."""
        two_f, h = gu.shape
        v = gu.view(two_f // (2 * G16), 2, G16, h)[:, which]

        def get():
            return v.reshape(two_f // 2, h)

        def set_(x):
            v.copy_(x.view(two_f // (2 * G16), G16, h))

        return get, set_

    @torch.no_grad()
    def init_random(self, seed: int = 0) -> None:
        """Deterministic partition-independent random init: the value of every global element
        depends only on (seed, logical name, global index) — any TP/PP/EP split of the same
        seed yields identical global weights (tests compare partitions against each other)."""
        std = self.cfg.init_std
        amp = std * math.sqrt(3.0)
        for lp in self.logical_params():
            if lp.split_dim is not None and lp.length == 0:
                continue
            if lp.init == "ones":
                lp.set(torch.ones(lp.local_shape(), dtype=self.dtype, device=self.device))
                continue
            if lp.init == "zeros":
                lp.set(torch.zeros(lp.local_shape(), dtype=self.dtype, device=self.device))
                continue
            shp = lp.local_shape()
            g = lp.global_shape
            if len(shp) == 1:
                buf = torch.empty(1, shp[0], dtype=self.dtype, device=self.device)
                ops.init_hash_(buf, 0, lp.offset if lp.split_dim == 0 else 0, g[0],
                               _name_seed(lp.name, seed), amp)
                lp.set(buf.view(shp))
                continue
            buf = torch.empty(shp, dtype=self.dtype, device=self.device)
            r0 = lp.offset if lp.split_dim == 0 else 0
            c0 = lp.offset if lp.split_dim == 1 else 0
            ops.init_hash_(buf, r0, c0, g[1], _name_seed(lp.name, seed), amp)
            lp.set(buf)
            del buf

    # ------------------------------------------------------------------------------------
    # forward
    # ------------------------------------------------------------------------------------
    def _norm(self, x, w, b, residual=None):
        if self.cfg.norm == "rms":
            return ops.rms_norm(x, w, self.cfg.norm_eps, residual=residual)
        return ops.layer_norm(x, w, b, self.cfg.norm_eps, residual=residual)

    def embed(self, fb: ForwardBatch) -> torch.Tensor:
        x = ops.embed(fb.input_ids, self.p["embed"], vstart=self.dims.vocab0)
        if self.tp > 1:
            self.comm.all_reduce_(x, "tp")
        if self.cfg.pos_emb == "learned":
            pe = ops.embed(fb.positions, self.p["pos_embed"], vstart=0)
            x = ops.add(x, pe)
        return x

    def forward(self, fb: ForwardBatch, kv_caches: Optional[list] = None,
                hidden_in: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Run this stage. Returns logits [R, vocab_local] on the last stage, else the
        residual stream [T, hidden] to send to the next stage."""
        if (self.seq_parallel and fb.is_prefill and fb.cp is None
                and fb.num_tokens >= max(self.sp_min_tokens, self.tp)):
            return self._forward_sp(fb, kv_caches, hidden_in)
        residual = self.embed(fb) if self.first else hidden_in
        if residual is None:
            raise ValueError("non-first pipeline stage needs hidden_in")
        if not self.first:
            residual = residual.clone()   # updated in place by the fused add+norm
        delta, partial = self._layers(fb, kv_caches, residual)
        if not self.last:
            if delta is None:
                return residual
            if partial:
                delta = self.comm.all_reduce_(delta, "tp")
            return ops.add(residual, ops.materialize(delta))
        idx = fb.logits_idx
        r = residual if idx is None else ops.gather_rows(residual, idx)
        if delta is not None:
            # all-reduce is linear: select the sampled rows first and reduce only those
            dl = delta if idx is None else ops.gather_rows(ops.materialize(delta), idx)
            if idx is None:
                r = r.clone()
            x = self._add_norm(dl, "final", r, partial)
        else:
            x = self._norm(r, self.p["final_w"], self.p.get("final_b"))
        return ops.linear(x, self.head_weight)

    def _layers(self, fb: ForwardBatch, kv_caches: Optional[list], residual: torch.Tensor) -> tuple:
        """This stage's layers over `residual` (updated in place by the fused add+norms).
        Returns the last FFN's output, still to be added: (delta, partial), `partial` meaning
        the TP all-reduce is pending too."""
        delta, partial = None, False      # FFN output of the previous layer (un-reduced if partial)
        for li, i in enumerate(self.layer_ids):
            pre = f"l{i}."
            if delta is None:
                x = self._norm(residual, self.p[pre + "in_w"], self.p.get(pre + "in_b"))
            else:
                x = self._add_norm(delta, pre + "in", residual, partial,
                                   consumer=(pre + "qkv_w", "bias" if pre + "qkv_b" in self.p else "none"))
            o = self._attention_block(li, pre, x, fb, kv_caches)
            route = None
            if (self.cfg.is_moe and self.tp == 1 and self.cfg.norm == "rms" and isinstance(o, ops.Partial)
                    and flags.get("BFLY_MOE_NORM_ROUTE")):
                # the add+RMSNorm routes the rows it normalises (one launch fewer per MoE layer)
                x, route = ops.rms_norm_route(o, self.p[pre + "post_w"], self.cfg.norm_eps, residual,
                                              self.p[pre + "router_w"], self.cfg.experts_per_token)
            else:
                x = self._add_norm(o, pre + "post", residual, self.tp > 1,
                                   consumer=(pre + "gu_w", "silu") if self.cfg.act == "silu" else None)
            delta, partial = self._ffn(pre, x, fb, route)
        return delta, partial

    def _attention_block(self, li: int, pre: str, x: torch.Tensor, fb: ForwardBatch,
                         kv_caches: Optional[list]):
        """normed x [T, h] -> QKV GEMM -> RoPE + KV append -> attention -> O GEMM (TP-partial)."""
        c, d = self.cfg, self.dims
        T, D = fb.num_tokens, c.head_dim
        kc, vc = kv_caches[li] if kv_caches is not None else (None, None)
        slots = fb.slots if kc is not None else None
        # split-K reduces are deferred into the consuming kernel (rope_kv / add+rmsnorm)
        # when no all-reduce sits in between (tp == 1)
        qkv = ops.linear(x, self.p[pre + "qkv_w"], bias=self.p.get(pre + "qkv_b"), defer=self.defer_qkv,
                         packed=self.packed.get(pre + "qkv_w"))
        if c.pos_emb == "rope":
            qkv = ops.rope_kv(qkv, fb.positions, self.cos, self.sin, d.hq, d.hkv, slots, kc, vc)
        elif kc is not None:
            k3 = qkv[:, d.hq * D:(d.hq + d.hkv) * D].view(T, d.hkv, D)
            v3 = qkv[:, (d.hq + d.hkv) * D:].view(T, d.hkv, D)
            ops.kv_append(k3, v3, fb.slots, kc, vc)
        q = qkv[:, : d.hq * D].view(T, d.hq, D)
        if fb.is_prefill:
            k = qkv[:, d.hq * D:(d.hq + d.hkv) * D].view(T, d.hkv, D)
            v = qkv[:, (d.hq + d.hkv) * D:].view(T, d.hkv, D)
            if fb.cp is not None:   # context parallel: ring (K/V circulate) or Ulysses
                from ..parallel import context_parallel as cpx

                fn = cpx.ulysses_attention if fb.cp.attn == "ulysses" else cpx.ring_attention
                sink = None
                if fb.cp.sink and kc is not None:   # this rank collects the prompt's K/V
                    sink = (lambda r, kk, vv, kc=kc, vc=vc:
                            ops.kv_append(kk.contiguous(), vv.contiguous(), fb.cp.sink[r], kc, vc))
                attn = fn(q, k, v, fb.cp, self.scale, sink)
            elif fb.num_decode or fb.prefix_lens is not None:
                attn = self._mixed_attention(q, k, v, fb, kc, vc)
            else:
                attn = ops.attn_prefill(q, k, v, fb.cu_seqlens, fb.max_seqlen, self.scale, True)
        else:
            attn = ops.attn_decode(q, kc, vc, fb.block_tables, fb.ctx_lens, self.scale, fb.max_ctx)
        return self._o_proj(pre, attn, T)

    def _o_proj(self, pre: str, attn: torch.Tensor, T: int):
        d, D = self.dims, self.cfg.head_dim
        o_b = self.p.get(pre + "o_b") if self.shard.tp_rank == 0 else None
        return ops.linear(attn.view(T, d.hq * D), self.p[pre + "o_w"], bias=o_b, defer=self.defer_reduce,
                          packed=self.packed.get(pre + "o_w"))

    # ------------------------------------------------------------------------------------
    # sequence parallelism (TP prefill)
    # ------------------------------------------------------------------------------------
    def _sp_pad(self, t: torch.Tensor, Tp: int) -> torch.Tensor:
        t = ops.materialize(t)
        if t.shape[0] == Tp:
            return t
        return torch.cat([t, t.new_zeros(Tp - t.shape[0], *t.shape[1:])])

    def _sp_scatter(self, t, Tp: int) -> torch.Tensor:
        """TP-partial [T, h] -> this rank's token shard [Tp / tp, h] of the sum (reduce-scatter)."""
        return self.comm.reduce_scatter(self._sp_pad(t, Tp), "tp")

    def _sp_gather(self, xs: torch.Tensor, T: int) -> torch.Tensor:
        """Token shards -> the full [T, h] activation on every TP rank (all-gather)."""
        return self.comm.all_gather(xs.contiguous(), "tp")[:T]

    def _forward_sp(self, fb: ForwardBatch, kv_caches: Optional[list],
                    hidden_in: Optional[torch.Tensor]) -> torch.Tensor:
        """forward() with the residual stream split by tokens over the TP group: rank r keeps
        rows [r * Ts, (r + 1) * Ts) (T padded to tp * Ts with zero rows, which stay zero
        through the norms). Every block: reduce-scatter the partial output into the shard,
        residual add + norm there, all-gather the normed rows for the next GEMM."""
        c = self.cfg
        T, tp = fb.num_tokens, self.tp
        Ts = (T + tp - 1) // tp
        Tp, r0 = Ts * tp, self.shard.tp_rank * Ts
        if self.first:
            # vocab-parallel embedding: each rank holds a partial sum of every row
            res = self._sp_scatter(ops.embed(fb.input_ids, self.p["embed"], vstart=self.dims.vocab0), Tp)
            if c.pos_emb == "learned":
                pos = self._sp_pad(fb.positions.view(-1, 1), Tp)[r0:r0 + Ts].view(-1)
                res = ops.add(res, ops.embed(pos, self.p["pos_embed"], vstart=0))
        else:
            if hidden_in is None:
                raise ValueError("non-first pipeline stage needs hidden_in")
            res = self._sp_pad(hidden_in, Tp)[r0:r0 + Ts].clone()
        delta = None
        for li, i in enumerate(self.layer_ids):
            pre = f"l{i}."
            w, b = self.p[pre + "in_w"], self.p.get(pre + "in_b")
            xs = self._norm(res, w, b) if delta is None else self._norm(self._sp_scatter(delta, Tp), w, b, residual=res)
            o = self._attention_block(li, pre, self._sp_gather(xs, T), fb, kv_caches)
            xs = self._norm(self._sp_scatter(o, Tp), self.p[pre + "post_w"], self.p.get(pre + "post_b"), residual=res)
            delta, _ = self._ffn(pre, self._sp_gather(xs, T), fb)
        if delta is not None:
            res = ops.add(res, self._sp_scatter(delta, Tp))
        full = self._sp_gather(res, T)
        if not self.last:
            return full
        if fb.logits_idx is not None:
            full = ops.gather_rows(full, fb.logits_idx)
        return ops.linear(self._norm(full, self.p["final_w"], self.p.get("final_b")), self.head_weight)

    def _mixed_attention(self, q, k, v, fb: ForwardBatch, kc, vc) -> torch.Tensor:
        """Attention of a mixed step: paged decode for the first num_decode rows; the prompt-
        chunk rows attend to their sequence's cached prefix and, causally, to the chunk itself.
        With a cached prefix that is ONE pass over the paged cache (ops.attn_prefill_paged: the
        chunk's K/V were appended by rope_kv just before), else flash attention over the chunk."""
        nd = fb.num_decode
        out = torch.empty(q.shape, dtype=q.dtype, device=q.device)   # both kernels write their rows
        if nd:
            ops.attn_decode(q[:nd], kc, vc, fb.block_tables, fb.ctx_lens, self.scale, fb.max_ctx, out=out[:nd])
        if q.shape[0] > nd:
            qp = q[nd:]
            if fb.split_seqs:
                # continuation chunks (leading): one paged pass over prefix + chunk; the fresh
                # prompts after them: flash attention over their own rows (2x the paged
                # kernel's rate on fresh prompts, profiles/r5_prof/)
                s1, r1 = fb.split_seqs, fb.split_rows
                ops.attn_prefill_paged(qp[:r1], kc, vc, fb.prefix_tables[:s1], fb.cu_seqlens[:s1 + 1],
                                       fb.positions[nd:nd + r1], fb.max_paged, self.scale, out=out[nd:nd + r1])
                ops.attn_prefill(qp[r1:], k[nd + r1:], v[nd + r1:], fb.cu_fresh, fb.max_fresh, self.scale, True,
                                 out=out[nd + r1:])
            elif fb.prefix_lens is not None and any(fb.prefix_lens):
                ops.attn_prefill_paged(qp, kc, vc, fb.prefix_tables, fb.cu_seqlens, fb.positions[nd:], fb.max_seqlen,
                                       self.scale, out=out[nd:])
            else:
                ops.attn_prefill(qp, k[nd:], v[nd:], fb.cu_seqlens, fb.max_seqlen, self.scale, True, out=out[nd:])
        return out

    def _add_norm(self, t: torch.Tensor, prefix: str, residual: torch.Tensor, partial: bool,
                  consumer: Optional[tuple] = None) -> torch.Tensor:
        """residual += (all_reduce(t) if partial else t); return norm(residual). With TP the
        all-reduce and the add+norm run as one fused kernel when the IPC all-reduce is on.
        `consumer` (weight name, epilogue): the GEMM that reads the result; on decode-sized
        batches whose plan takes a row scale, the norm returns an `ops.RowNormed`."""
        w, b = self.p[prefix + "_w"], self.p.get(prefix + "_b")
        if consumer is not None and not partial and 0 < residual.shape[0] <= self.rowscale_rows:
            cw = self.p[consumer[0]]
            if ops.rowscale_ok(residual.shape[0], cw.shape[0], cw.shape[1], consumer[1]):
                return ops.rms_norm(t, w, self.cfg.norm_eps, residual=residual, rows=True)
        if partial:
            if self.cfg.norm == "rms":
                return self.comm.all_reduce_rms_norm_(t, w, self.cfg.norm_eps, residual, "tp")
            t = self.comm.all_reduce_(t, "tp")
        return self._norm(t, w, b, residual=residual)

    def _ffn(self, pre: str, x: torch.Tensor, fb: ForwardBatch, route: Optional[tuple] = None) -> tuple:
        """Returns (out, partial): `partial` means `out` still needs the TP all-reduce, which
        the caller fuses with the next residual add + norm. `route`: (gates, topk_ids, topk_w)
        of a MoE layer already computed by the norm (ops.rms_norm_route)."""
        c, d = self.cfg, self.dims
        if c.is_moe:
            gates, topk_ids, topk_w = (route if route is not None else
                                       ops.moe_route(x, self.p[pre + "router_w"], c.experts_per_token))
            T = x.shape[0]
            # prefill: token-routed sparse experts (K12/K13: only routed rows are computed);
            # decode: dense fixed-shape path (weight-streaming bound either way, graph friendly)
            sparse = fb.is_prefill and self.device.type == "cuda" and flags.get("BFLY_MOE_SPARSE")
            if self.ep > 1 and fb.ep_alltoall and flags.get("BFLY_EP_ALLTOALL"):
                ipc = getattr(self.comm, "ep_ipc_prefill", None)
                if ipc is not None and ipc.fits(x, topk_ids, x.shape[0]):
                    return self._moe_ipc_prefill(pre, x, topk_ids, topk_w, ipc), False
                return self._moe_alltoall(pre, x, topk_ids, topk_w), False
            if self.ep > 1 and flags.get("BFLY_EP_DECODE_A2A"):
                # decode: graph-bucket padding rows (no cache slot) route nowhere
                return self._moe_alltoall_fixed(pre, x, topk_ids, topk_w, max(fb.ep_tokens, T),
                                                None if fb.is_prefill else fb.slots), False
            if self.ep > 1:
                # DP-attention + expert-parallel FFN: every EP rank contributes Tp rows (zero
                # padded), each computes its local experts on all ranks' tokens, and the
                # reduce-scatter returns each rank's own rows summed over experts.
                Tp = max(fb.ep_tokens, T)
                if Tp > T:
                    x = torch.cat([x, x.new_zeros(Tp - T, x.shape[1])])
                    gates = torch.cat([gates, gates.new_zeros(Tp - T, gates.shape[1])])
                    topk_ids = torch.cat([topk_ids, topk_ids.new_full((Tp - T, topk_ids.shape[1]), -1)])
                    topk_w = torch.cat([topk_w, topk_w.new_zeros(Tp - T, topk_w.shape[1])])
                xs = self.comm.all_gather(x, "ep")
                if sparse:
                    ids_s, w_s = self.comm.all_gather(topk_ids, "ep"), self.comm.all_gather(topk_w, "ep")
                else:
                    gs = self.comm.all_gather(gates, "ep")
            else:
                xs, gs, ids_s, w_s = x, gates, topk_ids, topk_w
            if sparse:
                out = ops.moe_sparse_ffn(xs, ids_s, w_s, self.p[pre + "moe_gu_w"], self.p[pre + "moe_down_w"],
                                         d.expert0, d.experts, d.ffn)
            else:
                if flags.get("BFLY_MOE_GATE_EPILOGUE"):   # routing weight in the GEMM epilogue
                    hmid = ops.linear_silu_gate(xs, self.p[pre + "moe_gu_w"], gs, d.expert0, d.experts,
                                                packed=self.packed.get(pre + "moe_gu_w"))
                else:
                    hmid = ops.linear(xs, self.p[pre + "moe_gu_w"], epilogue="silu")
                    ops.moe_gate_scale_(hmid, gs, d.expert0, d.experts)
                # one rank: the split-K reduce goes into the next add+RMSNorm, as for dense FFNs
                out = ops.linear(hmid, self.p[pre + "moe_down_w"], defer=self.defer_reduce and self.ep == 1,
                                 packed=self.packed.get(pre + "moe_down_w"))
            if self.ep > 1:
                return self.comm.reduce_scatter(out, "ep")[:T], False
            return out, self.tp > 1
        if c.act == "silu":
            hmid = ops.linear(x, self.p[pre + "gu_w"], epilogue="silu", packed=self.packed.get(pre + "gu_w"))
            out = ops.linear(hmid, self.p[pre + "down_w"], defer=self.defer_reduce, packed=self.packed.get(pre + "down_w"))
        else:
            hmid = ops.linear(x, self.p[pre + "fc_w"], bias=self.p.get(pre + "fc_b"))
            hmid = ops.gelu(hmid)
            pb = self.p.get(pre + "proj_b") if self.shard.tp_rank == 0 else None
            out = ops.linear(hmid, self.p[pre + "proj_w"], bias=pb)
        return out, self.tp > 1

    def _moe_alltoall(self, pre: str, x: torch.Tensor, topk_ids: torch.Tensor,
                      topk_w: torch.Tensor) -> torch.Tensor:
        """Expert-parallel MoE with token dispatch by all-to-all:
        each token travels only to the EP ranks that own one of its top-k experts (once per
        rank), the receiver runs its local experts on the routed rows (permute + grouped GEMM),
        and a second all-to-all returns the weighted partial outputs to be summed at the
        source. Used on steps where some EP rank prefills (variable-size exchange)."""
        d = self.dims
        T, H = x.shape
        k = topk_ids.shape[1]
        El, ep = d.experts, self.ep
        dest = torch.div(topk_ids.long().clamp(min=0), El, rounding_mode="floor").clamp(max=ep - 1)
        hit = torch.zeros(T, ep, dtype=torch.bool, device=x.device)
        if T:
            hit.scatter_(1, dest, True)
        r_idx, t_idx = hit.t().nonzero(as_tuple=True)        # grouped by destination rank
        splits = hit.sum(0).tolist()
        meta = torch.cat([topk_ids.float(), topk_w.float()], 1)[t_idx]   # ids exact in f32
        xr, rsplits = self.comm.all_to_all_v(x[t_idx], splits, "ep")
        mr, _ = self.comm.all_to_all_v(meta, splits, "ep")
        yr = ops.moe_sparse_ffn(xr, mr[:, :k].round().to(torch.int32).contiguous(), mr[:, k:].contiguous(),
                                self.p[pre + "moe_gu_w"], self.p[pre + "moe_down_w"], d.expert0, El, d.ffn)
        back, _ = self.comm.all_to_all_v(yr, rsplits, "ep")
        out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
        if T:
            out.index_add_(0, t_idx, back.float())
        return out.to(x.dtype)

    def _moe_ipc_prefill(self, pre: str, x: torch.Tensor, topk_ids: torch.Tensor, topk_w: torch.Tensor,
                         ipc) -> torch.Tensor:
        """Expert-parallel MoE on a prefill step without host synchronisation (VERDICT r3 item
        6): a device scan routes the tokens (counts, prefix sums, slots), each token row is
        stored once into every owning rank's IPC receive block with its local expert ids and
        weights, the per-source row counts travel in the receivers' headers, the receiver
        runs its grouped expert GEMMs over the rows that arrived (block counts bound the
        worst-case-sized buffer on the device), and only those rows return to be summed at
        the source in fixed rank order — the same values as the all-to-all path."""
        d = self.dims
        r = ipc.dispatch_prefill(x, topk_ids, topk_w, d.experts)
        yr = ops.moe_sparse_ffn(r.x, r.ids, r.w, self.p[pre + "moe_gu_w"], self.p[pre + "moe_down_w"], d.expert0,
                                d.experts, d.ffn, block_counts=(r.counts, r.cap))
        return ipc.combine(yr, r)

    def _moe_alltoall_fixed(self, pre: str, x: torch.Tensor, topk_ids: torch.Tensor,
                            topk_w: torch.Tensor, cap: int, slots: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Expert-parallel MoE over a FIXED-capacity all-to-all (decode; SURVEY.md §2.7-B B2,
        §3.2 (5)). Every EP rank reserves `cap` rows (the EP-agreed padded token count) per
        destination: a token goes once to each rank owning one of its top-k experts, at the
        position given by a running count over the tokens bound there, so no capacity can
        overflow and no token is dropped. Shapes are static and nothing waits on the host,
        so the layer replays inside the decode hipGraph. The exchange is comm.ep_dispatch /
        comm.ep_combine: byte-minimal over peer IPC buffers when enabled (parallel/ep_ipc.py:
        only routed rows travel, once each way), else ep_pack + all-to-all + ep_combine.
        The receiver computes ONLY routed rows (moe_align + grouped GEMMs skip padding, whose
        expert ids are -1); a second all-to-all brings each rank's weighted partial sums
        back, summed in f32 at the source.
        Link bytes equal the all-gather they replace; the MFMA work drops from ep x T rows
        of every local expert to the rows actually routed to it."""
        d = self.dims
        k = topk_ids.shape[1]
        r = self.comm.ep_dispatch(x, topk_ids, topk_w, slots, d.experts, cap)
        yr = ops.moe_sparse_ffn(r.x, r.ids, r.w, self.p[pre + "moe_gu_w"], self.p[pre + "moe_down_w"], d.expert0,
                                d.experts, d.ffn, expected_slots=cap * k)   # on average T x k routed slots per rank
        return self.comm.ep_combine(yr, r)

    # ------------------------------------------------------------------------------------
    # KV cache layout helpers
    # ------------------------------------------------------------------------------------
    def kv_bytes_per_token(self, dtype: Optional[torch.dtype] = None) -> int:
        """Local KV bytes per cached token (local layers x local kv heads x K,V)."""
        bits = torch.finfo(dtype or self.dtype).bits
        return 2 * len(self.layer_ids) * self.dims.hkv * self.cfg.head_dim * bits // 8

    def gemm_shapes(self) -> list:
        """(N, K) of every weight this stage multiplies by (workspace sizing)."""
        return sorted({tuple(w.shape) for k, w in self.p.items() if w.dim() == 2 and k != "embed"})

    def allocate_kv_cache(self, num_blocks: int, block_size: int, dtype: Optional[torch.dtype] = None) -> list:
        D, hk = self.cfg.head_dim, self.dims.hkv
        dt = dtype or self.dtype
        caches = []
        for _ in self.layer_ids:
            k = torch.zeros(num_blocks, hk, block_size, D, dtype=dt, device=self.device)
            v = torch.zeros(num_blocks, hk, D, block_size, dtype=dt, device=self.device)
            caches.append((k, v))
        return caches
