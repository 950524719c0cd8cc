"""Token selection over vocab-parallel logits.

Fast path (greedy and pure temperature sampling): the HIP sample kernel reduces each rank's
vocab shard to one (score, id) pair per row — Gumbel-max keyed on the GLOBAL token id and a
per-request seed, so shards are comparable — and the TP group all-gathers B x 8 bytes and
keeps the max (SURVEY.md §2.7-C "TP sampling"). No full-vocab gather, graph-capturable.

Filtered path (top-k / top-p): on the device, no host round trip, graph-capturable. Gumbel-max
restricted to a token subset samples the renormalised truncated distribution exactly, so
top-k / top-p reduce to one threshold per row on logit / temperature, passed to the same
kernel. The threshold comes from the row's global top-C candidates (C = 1024: each TP rank
takes its local top-C, the group all-gathers C values per row and keeps the global top-C) and
the global softmax normaliser (log-sum-exp all-gathered over TP):
  top-k : the k-th largest scaled logit (k > C is treated as C);
  top-p : among the candidates (after top-k), the last token whose preceding cumulative
          probability is <= p; if the candidates hold less than p of the mass the nucleus is
          truncated to them (a bounded nucleus of C tokens).
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
        pair = torch.stack([scores, ids.to(torch.float32)], 1)        # ids < 2^24: exact in f32
        allp = self.comm.all_gather(pair, "tp").view(self.tp, -1, 2)  # [tp, R, 2]
        best = allp[:, :, 0].argmax(0)                                 # ties -> lowest rank
        return allp.gather(0, best.view(1, -1, 1).expand(1, -1, 2))[0, :, 1].to(torch.int32)

    CANDIDATES = 1024

    def thresholds(self, lv: torch.Tensor, temps: torch.Tensor, params: list) -> torch.Tensor:
        """Per-row lower bound on logit / temperature implementing top-k / top-p (see module
        doc). Torch ops on the device plus two small TP all-gathers; no host sync."""
        R, Vl = lv.shape
        dev = lv.device
        t = temps.clamp(min=1e-6).view(R, 1)
        scaled = lv.float() / t
        # the same candidate count on every TP rank and for any split: min(C, whole vocab)
        C = min(self.CANDIDATES, self.vocab_size)
        vals = torch.topk(scaled, min(C, Vl), dim=1).values              # [R, <=C] descending
        if vals.shape[1] < C:                                            # small shard: pad
            vals = torch.cat([vals, vals.new_full((R, C - vals.shape[1]), float("-inf"))], 1)
        lse = torch.logsumexp(scaled, dim=1)
        if self.tp > 1:
            allv = self.comm.all_gather(vals.contiguous(), "tp").view(self.tp, R, C)
            vals = torch.topk(allv.permute(1, 0, 2).reshape(R, self.tp * C), C, dim=1).values
            lse = torch.logsumexp(self.comm.all_gather(lse.contiguous(), "tp").view(self.tp, R), 0)
        k = torch.tensor([min(p.top_k, C) if p.top_k > 0 else 0 for p in params], dtype=torch.long).to(dev)
        top_p = torch.tensor([p.top_p for p in params], dtype=torch.float32).to(dev)
        neg = torch.full((R,), float("-inf"), device=dev)
        has_k = k > 0
        thr_k = torch.where(has_k, vals.gather(1, (k - 1).clamp(min=0).view(R, 1)).view(R), neg)
        in_k = (~has_k).view(R, 1) | (torch.arange(C, device=dev).view(1, C) < k.view(R, 1))
        # top-p on the top-k-renormalised distribution (top-k applied first, as usual)
        den = torch.where(has_k, torch.logsumexp(vals.masked_fill(~in_k, float("-inf")), 1), lse)
        probs = torch.exp(vals - den.view(R, 1)).masked_fill(~in_k, 0.0)
        before = probs.cumsum(1) - probs                                 # mass ahead of each token
        drop = (before > top_p.view(R, 1)) | ~in_k
        last = torch.where(drop.any(1), drop.int().argmax(1) - 1, torch.full_like(k, C - 1)).clamp(min=0)
        thr_p = torch.where(top_p < 1.0, vals.gather(1, last.view(R, 1)).view(R), neg)
        thr = torch.maximum(thr_k, thr_p)
        # tolerance: the kernel scales by a reciprocal multiply, torch above by a division
        return thr - 1e-5 * thr.abs() - 1e-6

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
        pair = torch.stack([scores, ids.to(torch.float32)], 1)
        allp = self.comm.all_gather(pair, "tp").view(self.tp, -1, 2)
        best = allp[:, :, 0].argmax(0)
        return allp.gather(0, best.view(1, -1, 1).expand(1, -1, 2))[0, :, 1].to(torch.int32)
