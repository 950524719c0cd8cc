"""Token selection over vocab-parallel logits.

Fast path (greedy and pure temperature sampling): the HIP sample kernel reduces each rank's
vocab shard to one (score, id) pair per row — Gumbel-max keyed on the GLOBAL token id and a
per-request seed, so shards are comparable — and the TP group all-gathers B x 8 bytes and
keeps the max (SURVEY.md §2.7-C "TP sampling"). No full-vocab gather, graph-capturable.

Filtered path (top-k / top-p): on the device, no host round trip, graph-capturable. Gumbel-max
restricted to a token subset samples the renormalised truncated distribution exactly, so
top-k / top-p reduce to one threshold per row on logit / temperature, passed to the same
kernel. The threshold is EXACT: a radix select over the order-preserving 32-bit keys of the
scaled logits (ops.topkp_threshold, sample.hip tkp_*), 4 histogram passes of 8 bits per
filter, with every histogram SUM-all-reduced over the TP group so the vocab shards select
together. No candidate cap, no sort, no full-vocab gather:
  top-k : the k-th largest scaled logit (ties at it are kept);
  top-p : on the top-k-renormalised distribution, the smallest token value whose strictly
          larger tokens hold <= p of the mass (every token whose preceding mass is <= p).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import torch

from .. import ops


@dataclass
class SamplingParams:
    temperature: float = 0.0          # 0 = greedy
    top_k: int = 0                    # 0 = off
    top_p: float = 1.0
    max_tokens: int = 16
    stop_token_ids: list = field(default_factory=list)
    ignore_eos: bool = False
    seed: Optional[int] = None

    @property
    def needs_filter(self) -> bool:
        return self.temperature > 0 and (self.top_k > 0 or self.top_p < 1.0)


class Sampler:
    def __init__(self, comm, vocab_size: int, vocab_start: int, tp: int):
        self.comm = comm
        self.vocab_size = vocab_size
        self.vocab_start = vocab_start
        self.tp = tp

    def _local_valid(self, logits: torch.Tensor) -> torch.Tensor:
        # drop padded vocab rows (they exist so each shard is a multiple of 128 rows)
        n = max(0, min(logits.shape[1], self.vocab_size - self.vocab_start))
        return logits[:, :n]

    def sample(self, logits: torch.Tensor, temps: Optional[torch.Tensor] = None,
               seeds: Optional[torch.Tensor] = None, params: Optional[list] = None,
               check_finite: bool = False) -> torch.Tensor:
        """logits: [R, vocab_local]. Returns int32 token ids [R] (identical on every TP rank).
        `check_finite`: a row with an Inf / NaN logit on any TP rank samples -1 on every rank
        (the kernel scores it +inf, so it wins the TP merge)."""
        if params and any(p.needs_filter for p in params):
            return self._sample_filtered(logits, params, seeds, check_finite)
        lv = self._local_valid(logits)
        ids, scores = ops.sample(lv, temps, seeds, vstart=self.vocab_start, check_finite=check_finite)
        if self.tp == 1:
            return ids
        return self._merge(ids, scores)

    def _merge(self, ids: torch.Tensor, scores: torch.Tensor) -> torch.Tensor:
        """Each vocab shard's winner -> the global winner: (score, id) pairs all-gathered over
        the TP group, best score per row, lowest rank on ties (sample.hip pack / merge)."""
        allp = self.comm.all_gather(ops.sample_pack(scores, ids), "tp").view(self.tp, -1, 2)
        return ops.sample_merge(allp)

    def thresholds(self, lv: torch.Tensor, temps: torch.Tensor, params: list) -> torch.Tensor:
        """Per-row lower bound on logit / temperature implementing top-k / top-p (module doc).
        Radix-select kernels plus, under TP, one MAX and 4-8 SUM all-reduces of [R, 512]
        histograms; no host sync."""
        R = lv.shape[0]
        dev = lv.device
        top_k = torch.tensor([max(0, int(p.top_k)) for p in params], dtype=torch.int32).to(dev, non_blocking=True)
        top_p = torch.tensor([float(p.top_p) for p in params], dtype=torch.float32).to(dev, non_blocking=True)
        use_k = any(p.top_k > 0 and p.temperature > 0 for p in params)
        use_p = any(p.top_p < 1.0 and p.temperature > 0 for p in params)
        rsum = rmax = None
        if self.tp > 1:
            rsum = lambda t: self.comm.all_reduce_(t, "tp")          # noqa: E731
            rmax = lambda t: self.comm.all_reduce_max_(t, "tp")      # noqa: E731
        return ops.topkp_threshold(lv, temps, top_k, top_p, rsum, rmax, use_k, use_p)

    def _sample_filtered(self, logits, params, seeds, check_finite: bool = False):
        lv = self._local_valid(logits)
        R = lv.shape[0]
        temps = torch.tensor([p.temperature for p in params], dtype=torch.float32).to(lv.device)
        if seeds is None:
            seeds = torch.zeros(R, dtype=torch.int64, device=lv.device)
        thr = self.thresholds(lv, temps, params)
        ids, scores = ops.sample(lv, temps, seeds, vstart=self.vocab_start, thresh=thr.contiguous(),
                                 check_finite=check_finite)
        if self.tp == 1:
            return ids
        return self._merge(ids, scores)
