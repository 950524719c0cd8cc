"""Shard descriptors: which slice of the global model one rank owns.

A rank's shard is determined by its coordinates in the parallel mesh (PartitionPlan):
  * tensor parallel (tp): attention heads, FFN columns and the vocabulary are split
    (Megatron layout: QKV / gate-up column-parallel, O / down row-parallel);
  * pipeline parallel (pp): a contiguous layer range [layer_start, layer_end);
  * expert parallel (ep): a contiguous range of MoE experts.
All sizes here are pure functions of (ModelConfig, Shard) so every rank can compute every
other rank's layout (checkpoint resharding, partition planning) without communication.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

from ..config import ModelConfig


@dataclass(frozen=True)
class Shard:
    tp_rank: int = 0
    tp_size: int = 1
    layer_start: int = 0
    layer_end: Optional[int] = None   # None = all layers
    ep_rank: int = 0
    ep_size: int = 1
    num_layers_total: Optional[int] = None

    def layers(self, cfg: ModelConfig) -> range:
        end = cfg.num_layers if self.layer_end is None else self.layer_end
        return range(self.layer_start, end)

    def is_first(self, cfg: ModelConfig) -> bool:
        return self.layer_start == 0

    def is_last(self, cfg: ModelConfig) -> bool:
        return (cfg.num_layers if self.layer_end is None else self.layer_end) == cfg.num_layers


@dataclass(frozen=True)
class LocalDims:
    hq: int              # local query heads
    hkv: int             # local kv heads
    kv_head0: int        # first global kv head held locally
    q_head0: int
    ffn: int             # local FFN width (per expert for MoE)
    ffn0: int
    vocab: int           # local (padded) vocab rows
    vocab0: int
    vocab_padded: int    # global padded vocab
    experts: int         # local experts
    expert0: int


def vocab_padding_multiple(tp: int) -> int:
    # every local vocab shard is a multiple of 128 rows (GEMM N tiling)
    return 128 * tp


def local_dims(cfg: ModelConfig, s: Shard) -> LocalDims:
    tp, r = s.tp_size, s.tp_rank
    if cfg.num_heads % tp:
        raise ValueError(f"tp={tp} must divide num_heads={cfg.num_heads}")
    hq = cfg.num_heads // tp
    if cfg.num_kv_heads % tp == 0:
        hkv = cfg.num_kv_heads // tp
        kv0 = r * hkv
    elif tp % cfg.num_kv_heads == 0:
        hkv = 1                                   # kv heads replicated across tp ranks
        kv0 = r // (tp // cfg.num_kv_heads)
    else:
        raise ValueError(f"tp={tp} incompatible with num_kv_heads={cfg.num_kv_heads}")
    ffn_tp = tp if s.ep_size == 1 else 1         # EP shards experts, not their columns
    if cfg.intermediate_size % ffn_tp:
        raise ValueError("tp must divide intermediate_size")
    ffn = cfg.intermediate_size // ffn_tp
    ffn0 = (r if ffn_tp > 1 else 0) * ffn
    mult = vocab_padding_multiple(tp)
    vpad = (cfg.vocab_size + mult - 1) // mult * mult
    vl = vpad // tp
    if cfg.is_moe:
        if cfg.num_experts % s.ep_size:
            raise ValueError("ep must divide num_experts")
        el = cfg.num_experts // s.ep_size
        e0 = s.ep_rank * el
    else:
        el, e0 = 0, 0
    return LocalDims(hq=hq, hkv=hkv, kv_head0=kv0, q_head0=r * hq, ffn=ffn, ffn0=ffn0,
                     vocab=vl, vocab0=r * vl, vocab_padded=vpad, experts=el, expert0=e0)
